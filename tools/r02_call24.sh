# session 3 re-entry: full GPU suite + smoke + the default bench on HEAD
source tools/gpu_steps.sh
step 900 gpurun_out/r02_s3_gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 gpurun_out/r02_s3_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 900 gpurun_out/r02_s3_bench.log python -u bench.py
grep -h '^{' gpurun_out/r02_s3_bench.log > gpurun_out/r02_s3_bench.json
