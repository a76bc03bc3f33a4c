# ring scan + two tiles in flight pinned before the MFMAs (p2) vs ring (r3); parity of the tree (p2) first; diag split of p2
source tools/gpu_steps.sh
step 400 gpurun_out/r02_flat_p2_tests.log python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread
step 300 gpurun_out/r02_flatp_r3.log env ALAYA_AB_ROOT=$PWD/ab/r3 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatp_p2.log env ALAYA_AB_ROOT=$PWD/ab/p2 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatp_diag_p2.log env ALAYA_AB_ROOT=$PWD/ab/p2 python -u tools/flat_diag.py
grep -h "engine\|QPS" gpurun_out/r02_flatp_r3.log gpurun_out/r02_flatp_p2.log
