# early next-pop adjacency prefetch: search parity tests, then A/B kernel times vs the saved baseline
source tools/gpu_steps.sh
step 600 gpurun_out/r02_t21.log python -u -m pytest tests/test_gpu.py tests/test_sq8.py tests/test_updates.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step 600 gpurun_out/r02_ab21_new.log python -u tools/time_fixed.py --reps 30
ALAYA_AB_ROOT=$PWD/ab/base step 600 gpurun_out/r02_ab21_base.log python -u tools/time_fixed.py --reps 30
step 600 gpurun_out/r02_ab21_new2.log python -u tools/time_fixed.py --reps 30
grep -h "ms" gpurun_out/r02_ab21_*.log
