#!/bin/bash
# GPU-box script: the shard parity tests (f32 + SQ8, one batch and pipelined), then the N=2 bench
# shard path rehearsed on the one GPU over gloo (ALAYA_BENCH_REHEARSE=1) for config 4 and config 5
# shapes at reduced n.  Checks the code paths, not N-GPU numbers.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/shard_tests.log python -u -m pytest tests/test_shard_gpu.py tests/test_sq8.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
for wl in gist-hnsw sq8-ip; do
  ALAYA_BENCH_REHEARSE=1 step 600 gpurun_out/rehearse_$wl.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --workload $wl --n-base ${REHEARSE_N:-200000} --nq ${REHEARSE_NQ:-2000} --no-cpu-baseline --no-replica-leg
  grep '^{' gpurun_out/rehearse_$wl.log > gpurun_out/rehearse_$wl.json || true
done
