#!/bin/bash
# GPU-box script: the secondary configs on one MI355X with their CPU legs -- config 4's 10k-query batch
# (GIST-shaped), config 2 (flat MFMA scan) and config 3 (SIFT-shaped, 10k queries) -- JSON lines
# under gpurun_out/ (BASELINE.md §3).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/sec_c4_10k.log python -u bench.py --nq 10000 --steps 10 --warmup 2
grep '^{' gpurun_out/sec_c4_10k.log > gpurun_out/sec_c4_10k.json
step 600 gpurun_out/sec_c2_flat.log python -u bench.py --workload flat --steps 20 --warmup 3
grep '^{' gpurun_out/sec_c2_flat.log > gpurun_out/sec_c2_flat.json
step 600 gpurun_out/sec_c3_sift.log python -u bench.py --workload sift-hnsw --steps 20 --warmup 3
grep '^{' gpurun_out/sec_c3_sift.log > gpurun_out/sec_c3_sift.json
