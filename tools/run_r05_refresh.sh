#!/bin/bash
# GPU-box script (round 5): config 2 (flat) bench on the final tree (its line now cites the r05 PMC
# traffic), its rocprofv3 summary, and the headline's PMC traffic passes at ef 387 on the final tree.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r05_flat_final.log python -u bench.py --workload flat --steps 20 --warmup 3
grep '^{' gpurun_out/r05_flat_final.log > gpurun_out/r05_flat_final.json
step 300 gpurun_out/r05_flat_final_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flat_final -o run --output-format csv -- python bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
find gpurun_out/prof_flat_final -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r05_flat_final_kernel_stats.csv
rm -rf gpurun_out/prof_flat_final
EF=387 bash tools/run_pmc.sh gpurun_out/traffic_headline.json || exit $?
