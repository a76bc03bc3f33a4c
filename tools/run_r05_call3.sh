#!/bin/bash
# GPU-box script (round 5, call 3): helpers v2 (three requests per searcher, one memo) -- parity,
# the search suites with helpers forced on, then SIFT-shaped and config-5 A/B.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_helpers_tests.log python -u -m pytest tests/test_helpers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r05_helpers_tests.log && ! grep -q -E " failed| error" gpurun_out/r05_helpers_tests.log || exit 1
ALAYA_HELPERS=1 step 600 gpurun_out/r05_helpers_forced_suite.log python -u -m pytest tests/test_gpu.py tests/test_sq8.py tests/test_sq8_spill.py tests/test_operating_region.py tests/test_visited.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
step 300 gpurun_out/r05_help2_sift.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --envs="-,ALAYA_HELPERS=1,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=2,ALAYA_HELPERS=1+ALAYA_MAX_WAVES_PER_CU=8,-,ALAYA_HELPERS=1"
step 600 gpurun_out/r05_help2_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000,1250 --envs="-,ALAYA_HELPERS=1,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=1,-,ALAYA_HELPERS=1"
