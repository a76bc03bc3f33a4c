#!/bin/bash
# GPU-box script: (1) the stream-read calibration probe, (2) the one-GPU per-shard rehearsal of
# config 4 (tools/shard_rehearsal.py: G = 1, 2, 4, 8 shard graphs, 10k queries, predicted QPS),
# (3) the N = 2 bench shard path rehearsed on the one GPU over gloo for config 4 / config 5 shapes
# with the overlapped (ShardPipeline) and synchronous step times side by side.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
[ -n "$ONLY_REHEARSE" ] || step 120 gpurun_out/hbm_probe.log python -c "from alayalite_amd import _native; print('stream read GB/s', _native._ext.hbm_stream_read(0, 4 << 30, 5))"
[ -n "$ONLY_REHEARSE" ] || step 900 gpurun_out/shard_rehearsal.log python -u tools/shard_rehearsal.py --nq 10000 --out gpurun_out/shard_rehearsal_c4_10k.json
for wl in gist-hnsw sq8-ip; do
  ALAYA_BENCH_REHEARSE=1 step 600 gpurun_out/rehearse2_$wl.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 --workload $wl --n-base ${REHEARSE_N:-500000} --nq 10000 --no-cpu-baseline --no-replica-leg
  grep '^{' gpurun_out/rehearse2_$wl.log > gpurun_out/rehearse2_$wl.json || true
done
