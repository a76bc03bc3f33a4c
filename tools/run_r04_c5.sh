#!/bin/bash
# GPU-box script (round 4): config 5 at its full batch on the spill-table kernel -- bench with the
# recall sweep and the CPU leg, the rocprofv3 kernel summary at the chosen ef, per-phase stamps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r04_c5_10k.log python -u bench.py --workload sq8-ip --nq 10000 --steps 20 --warmup 3
grep '^{' gpurun_out/r04_c5_10k.log > gpurun_out/r04_c5_10k.json
EF=$(python -c "import json; print(json.load(open('gpurun_out/r04_c5_10k.json'))['config']['ef_search'])")
echo "ef=$EF"
step 900 gpurun_out/r04_c5_10k_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python -u bench.py --workload sq8-ip --nq 10000 --ef $EF --steps 20 --warmup 3 --no-cpu-baseline
find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r04_c5_10k_kernel_stats.csv
rm -rf gpurun_out/prof_c5
step 900 gpurun_out/r04_c5_phases.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --dim 768 --nq 10000 --ef $EF --builder gpu
