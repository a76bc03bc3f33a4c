source tools/gpu_steps.sh
step 900 gpurun_out/r02_tests1.log python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider
step 120 gpurun_out/r02_smoke1.log python -c "import __graft_entry__ as g; g.smoke()"
step 600 gpurun_out/r02_bench1.log python -u bench.py --steps 20 --warmup 5
