# ring scan + consumer-side wave prefilter mask (pf) vs ring (r3); parity of the tree (pf) first
source tools/gpu_steps.sh
step 400 gpurun_out/r02_flat_pf_tests.log python -u -m pytest tests/test_flat.py -m gpu -x -q --timeout 120 --timeout-method thread
step 300 gpurun_out/r02_flatpf_r3.log env ALAYA_AB_ROOT=$PWD/ab/r3 python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatpf_pf.log env ALAYA_AB_ROOT=$PWD/ab/pf python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatpf_diag.log env ALAYA_AB_ROOT=$PWD/ab/pf python -u tools/flat_diag.py
grep -h "engine\|QPS" gpurun_out/r02_flatpf_r3.log gpurun_out/r02_flatpf_pf.log
