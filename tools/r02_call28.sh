# flat scan: ring-decoupled warp specialisation (r2: 2 slots, 80-entry buffers; r3: 3 slots, 64) vs base;
# parity tests of the in-tree build (r3) first
source tools/gpu_steps.sh
step 400 gpurun_out/r02_flat_r3_tests.log python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread
step 300 gpurun_out/r02_flatring_base.log env ALAYA_AB_ROOT=$PWD/ab/base python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatring_r2.log env ALAYA_AB_ROOT=$PWD/ab/r2 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatring_r3.log env ALAYA_AB_ROOT=$PWD/ab/r3 python -u tools/ab_flat.py --dims 128,64,224
grep -h "engine\|QPS" gpurun_out/r02_flatring_*.log
