#!/bin/bash
# GPU-box script mirroring the driver's round end on one GPU: parity suite, smoke(), the default
# bench (N = 1, CPU leg) + its rocprofv3 kernel summary at the chosen ef (tools/run_final.sh), then
# the driver's N = 2 command with both ranks on this GPU over gloo (ALAYA_BENCH_REHEARSE=1, default
# workload, replica leg included) -- a check of the multi-GPU code path, not a scaling number.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/run_final.sh || exit $?
source tools/gpu_steps.sh
ALAYA_BENCH_REHEARSE=1 step 900 gpurun_out/rehearse2_default.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2
grep '^{' gpurun_out/rehearse2_default.log > gpurun_out/rehearse2_default.json
