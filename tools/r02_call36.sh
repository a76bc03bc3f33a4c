# final tree: GPU suite, smoke, default bench (headline) and its rocprof kernel stats
source tools/gpu_steps.sh
step 900 gpurun_out/r02_final_gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 gpurun_out/r02_final_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 900 gpurun_out/r02_final_bench.log python -u bench.py
grep -h '^{' gpurun_out/r02_final_bench.log > gpurun_out/r02_final_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 600 gpurun_out/r02_final_bench_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
