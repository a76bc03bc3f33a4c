source tools/gpu_steps.sh
step 600 gpurun_out/r02_flat_tests8.log python -u -m pytest tests/test_flat.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step 400 gpurun_out/r02_flat_bench960.log python -u bench.py --workload flat --dim 960 --steps 10 --warmup 3 --no-cpu-baseline
step 400 gpurun_out/r02_flat_bench768.log python -u bench.py --workload flat --dim 768 --steps 10 --warmup 3 --no-cpu-baseline
