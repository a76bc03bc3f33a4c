#!/bin/bash
# GPU-box script: the N=2 shard-mode bench path (torchrun, 2 ranks) rehearsed on the one GPU of the
# box with gloo (ALAYA_BENCH_REHEARSE=1).  Checks the code path, not the N-GPU numbers.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ALAYA_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --n-base 200000 --no-cpu-baseline > gpurun_out/rehearse.json 2> gpurun_out/rehearse.log || { tail -40 gpurun_out/rehearse.log; exit 1; }
cat gpurun_out/rehearse.json
grep "\[bench\]" gpurun_out/rehearse.log | tail -5
