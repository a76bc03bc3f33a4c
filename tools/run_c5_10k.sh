#!/bin/bash
# GPU-box script: config 5 at its full batch on one MI355X (10M x 768 IP, SQ8 search + reference
# rerank, 10k queries, ef fixed at the operating point), then the rocprofv3 kernel summary of the
# same command.  Logs/JSON under gpurun_out/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
EF=${EF:-340}
step 600 gpurun_out/c5_10k.log python -u bench.py --workload sq8-ip --nq 10000 --ef $EF --steps 20 --warmup 3
grep '^{' gpurun_out/c5_10k.log > gpurun_out/c5_10k.json
step 600 gpurun_out/c5_10k_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_10k -o run --output-format csv -- python -u bench.py --workload sq8-ip --nq 10000 --ef $EF --steps 20 --warmup 3 --no-cpu-baseline --no-tail-probe
find gpurun_out/prof_c5_10k -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/c5_10k_kernel_stats.csv
rm -f gpurun_out/prof_c5_10k/*/*kernel_trace.csv gpurun_out/prof_c5_10k/*kernel_trace.csv
cut -c1-160 gpurun_out/c5_10k_kernel_stats.csv | head -6
