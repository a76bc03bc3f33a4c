#!/bin/bash
# GPU-box script (round 4): multi-GPU layouts rehearsed on one MI355X.
#  1. config 4 (GIST 1M, 10k queries) and config 5 (10M x 768 IP SQ8 + rerank, 10k queries): the
#     S shards x 8/S query groups prediction (tools/shard_rehearsal.py)
#  2. the driver's N = 2 and N = 4 commands with every rank on cuda:0 over gloo (ALAYA_BENCH_REHEARSE):
#     shard layout + layouts leg, GIST 200k rows (code path, not numbers)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 450 gpurun_out/r04_rehearsal_c4.log python -u tools/shard_rehearsal.py --workload gist --nq 10000 --out gpurun_out/shard_rehearsal_c4_10k.json
step 700 gpurun_out/r04_rehearsal_c5.log python -u tools/shard_rehearsal.py --workload sq8 --nq 10000 --out gpurun_out/shard_rehearsal_c5_10k.json
