#!/bin/bash
# GPU-box script (round 4): f32 rows on the spill table (kSpace 3) -- parity, then config 3 (SIFT 1M,
# 10k / 1k queries) LDS first level vs the spill table, residency 16 / 20 searchers per CU.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/r04_sift_tests.log python -u -m pytest tests/test_visited.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread --maxfail 4
grep -q " passed" gpurun_out/r04_sift_tests.log && ! grep -q " failed" gpurun_out/r04_sift_tests.log || exit 1
step 600 gpurun_out/r04_sift_ab.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --max-waves 16,20 --table 0,-7 --envs "-,ALAYA_SPILL_TABLE_F32=1+ALAYA_VIS_LIMIT=1,ALAYA_SPILL_TABLE_F32=1"
