#!/bin/bash
# GPU-box script (round 4): the overlay descent in its own launch (hnsw_descent_kernel, one-trip hops
# on (id, offset) pairs) -- the GPU suite, then SIFT / config 5 / GIST-1k A/B against the inline
# descent (ALAYA_INLINE_DESCENT=1) and the two-trip descent kernel (ALAYA_NO_UPPER_PAIRS=1).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/r04_descent_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/r04_descent_suite.log && ! grep -q " failed" gpurun_out/r04_descent_suite.log || exit 1
step 300 gpurun_out/r04_descent_sift.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --envs="-,ALAYA_INLINE_DESCENT=1,ALAYA_NO_UPPER_PAIRS=1,-,ALAYA_INLINE_DESCENT=1"
step 300 gpurun_out/r04_descent_gist.log python -u tools/shape_sweep.py --workload gist --nq 1000,10000 --envs="-,ALAYA_INLINE_DESCENT=1,-,ALAYA_INLINE_DESCENT=1"
step 600 gpurun_out/r04_descent_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --envs="-,ALAYA_INLINE_DESCENT=1,ALAYA_NO_UPPER_PAIRS=1,-,ALAYA_INLINE_DESCENT=1"
