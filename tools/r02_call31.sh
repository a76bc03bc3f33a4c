# flat ring + producer-side threshold masks (m3) vs ring (r3) vs base; parity of the tree (m3) first
source tools/gpu_steps.sh
step 400 gpurun_out/r02_flat_m3_tests.log python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread
step 300 gpurun_out/r02_flatm_base.log env ALAYA_AB_ROOT=$PWD/ab/base python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatm_r3.log env ALAYA_AB_ROOT=$PWD/ab/r3 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatm_m3.log env ALAYA_AB_ROOT=$PWD/ab/m3 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatm_diag_m3.log env ALAYA_AB_ROOT=$PWD/ab/m3 python -u tools/flat_diag.py
grep -h "engine\|QPS" gpurun_out/r02_flatm_*.log
