#!/bin/bash
# GPU-box script (round 4, final tree after the flat two-ahead tiles): parity suite, smoke, default
# bench + rocprof (tools/run_final.sh), then config 2 (flat) and config 4's 10k batch with CPU legs.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/run_final.sh || exit $?
source tools/gpu_steps.sh
step 600 gpurun_out/sec_c2_flat.log python -u bench.py --workload flat --steps 20 --warmup 3
grep '^{' gpurun_out/sec_c2_flat.log > gpurun_out/sec_c2_flat.json
step 600 gpurun_out/sec_c4_10k.log python -u bench.py --nq 10000 --steps 10 --warmup 2
grep '^{' gpurun_out/sec_c4_10k.log > gpurun_out/sec_c4_10k.json
