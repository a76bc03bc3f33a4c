# pool-distance register mirror (m0: f32 rows <= 8 chunks only; m6: + SQ8 with 6 registers) vs base; parity of the tree (m6) first
source tools/gpu_steps.sh
PYTHONPATH=$PWD/ab/m6:$PWD step 60 gpurun_out/r02_mir_which.log python -c "import alayalite_amd._native as n; print(n.__file__)"
PYTHONPATH=$PWD/ab/m6:$PWD step 600 gpurun_out/r02_mir_tests.log python -u -m pytest tests/test_gpu.py tests/test_sq8.py tests/test_golden.py tests/test_updates.py tests/test_operating_region.py tests/test_contracts_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step 600 gpurun_out/r02_mir_base.log env ALAYA_AB_ROOT=$PWD/ab/base python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
step 600 gpurun_out/r02_mir_m0.log env ALAYA_AB_ROOT=$PWD/ab/m0 python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
step 600 gpurun_out/r02_mir_m6.log env ALAYA_AB_ROOT=$PWD/ab/m6 python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
step 600 gpurun_out/r02_mir_base2.log env ALAYA_AB_ROOT=$PWD/ab/base python -u tools/time_fixed.py --reps 20 --only sift,sift1k,sq8
grep -H " ms" gpurun_out/r02_mir_*.log
