#!/bin/bash
# GPU-box script (round 5): config 4's N = 8 layouts rehearsed on one MI355X with the round-5 kernels
# (two waves per SIMD past residency, helpers), per-rank breakdown; then the PMC traffic passes of
# config 5 at 10k queries (ef 368) on the current kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 500 gpurun_out/r05_rehearsal_c4.log python -u tools/shard_rehearsal.py --workload gist --nq 10000 --out gpurun_out/shard_rehearsal_c4_10k.json
EF=368 bash tools/run_pmc.sh gpurun_out/traffic_sq8_c5_10k.json --workload sq8-ip --nq 10000 || exit $?
