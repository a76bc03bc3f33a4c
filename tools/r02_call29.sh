# flat ring variants: r3 (3 slots, kB 64), r3p (+ row norms a tile ahead), r4p (4 slots, kB 48, + norms ahead); diag split of r3p
source tools/gpu_steps.sh
step 300 gpurun_out/r02_flatring2_r3.log env ALAYA_AB_ROOT=$PWD/ab/r3 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatring2_r3p.log env ALAYA_AB_ROOT=$PWD/ab/r3p python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatring2_r4p.log env ALAYA_AB_ROOT=$PWD/ab/r4p python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatring2_diag_r3p.log env ALAYA_AB_ROOT=$PWD/ab/r3p python -u tools/flat_diag.py
step 400 gpurun_out/r02_flat_r4p_tests.log python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread
grep -h "engine\|QPS" gpurun_out/r02_flatring2_r*.log
