source tools/gpu_steps.sh
step 600 gpurun_out/r02_flat_tests14.log python -u -m pytest tests/test_flat.py tests/test_contracts_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step 300 gpurun_out/r02_flat_ws.log python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
ALAYA_FLAT_WS0=1 step 300 gpurun_out/r02_flat_old.log python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
grep -h '^{' gpurun_out/r02_flat_ws.log gpurun_out/r02_flat_old.log | python -c "import sys, json; [print(json.loads(l)['value'], json.loads(l)['roofline']['kernel_ms'], json.loads(l)['roofline']['frac'], json.loads(l)['config']['flagged_queries']) for l in sys.stdin]"
