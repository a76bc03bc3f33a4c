#!/bin/bash
# GPU-box script (round 5): config 5's N = 8 layouts rehearsed on one MI355X with the round-5 kernels.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r05_rehearsal_c5.log python -u tools/shard_rehearsal.py --workload sq8 --nq 10000 --out gpurun_out/shard_rehearsal_c5_10k.json
