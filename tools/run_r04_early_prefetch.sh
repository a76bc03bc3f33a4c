#!/bin/bash
# GPU-box script (round 4): the second-level prefetch issued right after the first row pass --
# parity (forced-spill SQ8 suite, visited, SQ8), then config 5 with the prefetch early (default) and
# after a wait for the rows (ALAYA_SPILL_FLAGS=4), and the first-level policy.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r04_ep_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_visited.py tests/test_sq8.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread --maxfail 4
grep -q " passed" gpurun_out/r04_ep_tests.log && ! grep -q " failed" gpurun_out/r04_ep_tests.log || exit 1
step 900 gpurun_out/r04_ep_c5.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000 --ef 368 --envs="-,ALAYA_SPILL_FLAGS=4"
