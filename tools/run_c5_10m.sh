#!/bin/bash
# GPU-box script: BASELINE config 5 at full size on one MI355X -- 10M x 768 IP, SQ8 search + f32
# rerank, graph from the device build -- then the rocprofv3 kernel summary at the chosen ef.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py --workload sq8-ip --steps 20 --warmup 3 > gpurun_out/bench_c5_10m.json 2> gpurun_out/bench_c5_10m.log || { tail -30 gpurun_out/bench_c5_10m.log; exit 1; }
cat gpurun_out/bench_c5_10m.json
EF=$(python -c "import json;print(json.load(open('gpurun_out/bench_c5_10m.json'))['config']['ef_search'])")
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python -u bench.py --workload sq8-ip --ef $EF --steps 20 --warmup 3 --no-cpu-baseline --no-tail-probe > gpurun_out/bench_c5_prof.json 2> gpurun_out/bench_c5_prof.log || { tail -20 gpurun_out/bench_c5_prof.log; exit 1; }
cut -c1-200 gpurun_out/prof_c5/run_kernel_stats.csv | head -8
