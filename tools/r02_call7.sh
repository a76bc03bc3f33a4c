source tools/gpu_steps.sh
step 600 gpurun_out/r02_flat_tests.log python -u -m pytest tests/test_flat.py tests/test_contracts_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step 300 gpurun_out/r02_flat_bench.log python -u bench.py --workload flat --steps 10 --warmup 3 --no-cpu-baseline
step 300 gpurun_out/r02_flat_bench960.log python -u bench.py --workload flat --dim 960 --steps 10 --warmup 3 --no-cpu-baseline
step 900 gpurun_out/r02_tests7.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
