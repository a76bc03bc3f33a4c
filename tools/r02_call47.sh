# final build: smoke and the default bench
source tools/gpu_steps.sh
step 300 gpurun_out/r02_fin_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 900 gpurun_out/r02_fin_bench.log python -u bench.py
grep -h '^{' gpurun_out/r02_fin_bench.log > gpurun_out/r02_fin_bench.json
