#!/bin/bash
# one GPU call after a search-kernel change: parity suite, config 3 bench + rocprof, launch-shape
# sweeps of the three graph workloads, SQ counters of SIFT at 10k queries
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q " failed" gpurun_out/gpu_suite.log || exit 1
step 600 gpurun_out/c3.log python -u bench.py --workload sift-hnsw --steps 20 --warmup 3
grep '^{' gpurun_out/c3.log > gpurun_out/c3.json
EF=$(python -c "import json;print(json.load(open('gpurun_out/c3.json'))['config']['ef_search'])")
step 600 gpurun_out/c3_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python -u bench.py --workload sift-hnsw --ef $EF --steps 20 --warmup 3 --no-cpu-baseline
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c3_kernel_stats.csv
find gpurun_out/prof_c3 -name "*kernel_trace.csv" -delete
step 300 gpurun_out/sw_sift.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --max-waves 0,20
step 300 gpurun_out/sw_gist.log python -u tools/shape_sweep.py --workload gist --nq 1000,10000
step 400 gpurun_out/sw_sq8.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
WORKLOAD=sift NQ=10000 EF=70 bash tools/run_pmc_sq.sh
