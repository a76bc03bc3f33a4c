#!/bin/bash
# GPU-box script (round 5, final tree): the whole -m gpu suite, smoke(), the default bench (headline,
# GIST 1M / 1k) + its rocprofv3 summary, config 3 (SIFT-shaped 1M / 10k) and config 5 (10M x 768 IP
# SQ8 + rerank / 10k) benches with their rocprofv3 summaries.  Logs under gpurun_out/r05f_*.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r05f_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step 300 gpurun_out/r05f_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
bash tools/run_bench_1m.sh || exit $?
cat gpurun_out/bench_1m.json
find gpurun_out/prof_1m -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r05f_headline_kernel_stats.csv
rm -f gpurun_out/prof_1m/*kernel_trace.csv gpurun_out/prof_1m/*/*kernel_trace.csv
step 600 gpurun_out/r05f_c3.log python -u bench.py --workload sift-hnsw --nq 10000 --steps 20 --warmup 3
grep '^{' gpurun_out/r05f_c3.log > gpurun_out/r05f_c3.json
EF=$(python -c "import json;print(json.load(open('gpurun_out/r05f_c3.json'))['config']['ef_search'])")
step 400 gpurun_out/r05f_c3_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05f_c3 -o run --output-format csv -- python -u bench.py --workload sift-hnsw --nq 10000 --ef $EF --steps 20 --warmup 3 --no-cpu-baseline --no-tail-probe
find gpurun_out/prof_r05f_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r05f_c3_kernel_stats.csv
rm -rf gpurun_out/prof_r05f_c3
EF=368 bash tools/run_c5_10k.sh || exit $?
