# round-2 headline evidence: default bench (as the driver runs it), its rocprofv3 kernel stats,
# and the PMC traffic passes at the same operating point (device-built graph: deterministic ef)
source tools/gpu_steps.sh
export TMPDIR=/tmp
step 600 gpurun_out/r02_bench_default.log python -u bench.py --steps 20 --warmup 5
grep '^{' gpurun_out/r02_bench_default.log > gpurun_out/r02_bench_default.json
EF=$(python -c "import json; print(json.load(open('gpurun_out/r02_bench_default.json'))['config']['ef_search'])")
echo "operating ef $EF"
step 600 gpurun_out/r02_bench_rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --ef $EF --no-cpu-baseline
EF=$EF timeout -k 10 900 bash tools/run_pmc.sh > gpurun_out/r02_pmc.log 2>&1; echo "pmc rc=$?"
tail -3 gpurun_out/r02_pmc.log
