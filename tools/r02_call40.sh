# L2 warm-up of the predicted next expansion's neighbour rows (ALAYA_PF_ROWS=1) vs off, same build;
# parity of the search tests with it on first
source tools/gpu_steps.sh
ALAYA_PF_ROWS=1 step 600 gpurun_out/r02_pf_tests.log python -u -m pytest tests/test_gpu.py tests/test_sq8.py tests/test_golden.py tests/test_updates.py tests/test_operating_region.py -m gpu -x -q --timeout 200 --timeout-method thread
ALAYA_PF_ROWS=0 step 600 gpurun_out/r02_pf_off.log python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
ALAYA_PF_ROWS=1 step 600 gpurun_out/r02_pf_on.log python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
ALAYA_PF_ROWS=0 step 600 gpurun_out/r02_pf_off2.log python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
grep -H "ms" gpurun_out/r02_pf_off.log gpurun_out/r02_pf_on.log gpurun_out/r02_pf_off2.log
