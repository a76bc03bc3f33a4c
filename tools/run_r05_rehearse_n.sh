#!/bin/bash
# GPU-box script (round 5): bench.py's N-rank path with every rank on cuda:0 over gloo -- N = 2 and
# N = 4 (shard layout, then the layouts leg), GIST-shaped 200k rows, with the search on a
# CU-reserving stream (--exchange-cus 8, the RCCL default) so the masked-stream pipeline runs in the
# driver's command shape; then N = 2 on config 5's workload shape.  Checks the code, not the numbers.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export ALAYA_BENCH_REHEARSE=1
source tools/gpu_steps.sh
step 600 gpurun_out/r05_rehearse2_gist.log python -u bench.py --gpus 2 --n 200000 --nq 2000 --steps 5 --warmup 1 --exchange-cus 8
grep '^{' gpurun_out/r05_rehearse2_gist.log > gpurun_out/r05_rehearse2_gist.json
step 600 gpurun_out/r05_rehearse4_gist.log python -u bench.py --gpus 4 --n 200000 --nq 2000 --steps 5 --warmup 1 --exchange-cus 8
grep '^{' gpurun_out/r05_rehearse4_gist.log > gpurun_out/r05_rehearse4_gist.json
step 900 gpurun_out/r05_rehearse2_sq8.log python -u bench.py --gpus 2 --workload sq8-ip --n 1000000 --nq 2000 --steps 5 --warmup 1 --exchange-cus 8
grep '^{' gpurun_out/r05_rehearse2_sq8.log > gpurun_out/r05_rehearse2_sq8.json
