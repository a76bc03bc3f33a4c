#!/bin/bash
# GPU-box script (round 4, final tree): config 5 at 10k queries (bench + rocprof at its ef), then
# config 3 (SIFT-shaped) and config 2 (flat) with their CPU legs.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
EF=368 bash tools/run_c5_10k.sh || exit $?
source tools/gpu_steps.sh
step 600 gpurun_out/sec_c3_sift.log python -u bench.py --workload sift-hnsw --steps 20 --warmup 3
grep '^{' gpurun_out/sec_c3_sift.log > gpurun_out/sec_c3_sift.json
step 600 gpurun_out/sec_c2_flat.log python -u bench.py --workload flat --steps 20 --warmup 3
grep '^{' gpurun_out/sec_c2_flat.log > gpurun_out/sec_c2_flat.json
