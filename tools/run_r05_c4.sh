#!/bin/bash
# GPU-box script (round 5): config 4's batch (GIST-shaped 1M, 10k queries) on one GPU on the final
# tree, with the CPU leg, and the rocprofv3 summary of the same command.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/r05_c4_10k.log python -u bench.py --nq 10000 --steps 10 --warmup 2
grep '^{' gpurun_out/r05_c4_10k.log > gpurun_out/r05_c4_10k.json
EF=$(python -c "import json;print(json.load(open('gpurun_out/r05_c4_10k.json'))['config']['ef_search'])")
step 400 gpurun_out/r05_c4_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_c4 -o run --output-format csv -- python -u bench.py --nq 10000 --ef $EF --steps 10 --warmup 2 --no-cpu-baseline --no-tail-probe
find gpurun_out/prof_r05_c4 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r05_c4_kernel_stats.csv
rm -rf gpurun_out/prof_r05_c4
