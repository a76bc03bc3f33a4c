#!/bin/bash
# GPU-box script (round 5, call 6): wave placement probe; GIST-shaped batches around the 1,024
# resident searchers of the d = 960 kernel (config 4's S = 1 layout runs 1,250 per rank) on the tree
# and on a 2-waves-per-SIMD build (ab/wide1: one row per lane group); the RCCL exchange beside the
# search with and without reserved CUs; the single-rank RCCL tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 60 gpurun_out/r05_simd_probe.log ./tools/simd_probe
step 600 gpurun_out/r05_gist_rounds.log python -u tools/shape_sweep.py --workload gist --ef 373 --nq 1000,1024,1250,2048,10000
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/wide1 step 600 gpurun_out/r05_gist_rounds_wide1.log python -u tools/shape_sweep.py --workload gist --ef 373 --nq 1000,1024,1250,2048,10000
step 300 gpurun_out/r05_rccl_tests.log python -u -m pytest tests/test_shard_gpu.py -q -p no:cacheprovider --timeout 240 --timeout-method thread
step 600 gpurun_out/r05_rccl_overlap.log python -u tools/rccl_overlap.py --workload gist --nq 10000 --steps 10 --reserve 0,8,16 --out gpurun_out/r05_rccl_overlap.json
