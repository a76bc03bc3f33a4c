#!/bin/bash
# GPU-box script (round 4): bench lines with the batch_tail figure -- the headline, config 3, config 5.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/tb_default.log python -u bench.py --steps 20 --warmup 3
grep '^{' gpurun_out/tb_default.log > gpurun_out/tb_default.json
step 600 gpurun_out/tb_sift.log python -u bench.py --workload sift-hnsw --steps 20 --warmup 3
grep '^{' gpurun_out/tb_sift.log > gpurun_out/tb_sift.json
step 600 gpurun_out/tb_c5.log python -u bench.py --workload sq8-ip --nq 10000 --ef 368 --steps 20 --warmup 3
grep '^{' gpurun_out/tb_c5.log > gpurun_out/tb_c5.json
