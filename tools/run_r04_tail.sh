#!/bin/bash
# GPU-box script (round 4): tail share of the latency-bound batches (tools/tail_probe.py), SIFT then
# config 5, plus the 1M flat parity test at config 2's size.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r04_tail_sift.log python -u tools/tail_probe.py --workload sift
step 300 gpurun_out/r04_flat1m.log python -u -m pytest tests/test_flat.py -q -p no:cacheprovider --timeout 240 --timeout-method thread -k 1m
step 600 gpurun_out/r04_tail_sq8.log python -u tools/tail_probe.py --workload sq8 --pre-ef 20,40
