#!/bin/bash
# GPU-box script (round 4): tail helpers (ALAYA_SPILL_FLAGS=32: a wave with no query left warms L2
# for a sibling's predicted next expansion) -- parity with helpers on, then config 5 and SIFT (4-wave
# workgroups) A/B, and the pre-change build (ab/base).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
ALAYA_SPILL_FLAGS=32 step 400 gpurun_out/r04_helper_tests.log python -u -m pytest tests/test_sq8.py tests/test_sq8_spill.py tests/test_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r04_helper_tests.log && ! grep -q " failed" gpurun_out/r04_helper_tests.log || exit 1
step 600 gpurun_out/r04_helper_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --envs="-,ALAYA_SPILL_FLAGS=32,-,ALAYA_SPILL_FLAGS=32"
step 300 gpurun_out/r04_helper_sift.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --envs="-,ALAYA_SEARCH_WAVES=4,ALAYA_SEARCH_WAVES=4+ALAYA_SPILL_FLAGS=32,-,ALAYA_SEARCH_WAVES=4,ALAYA_SEARCH_WAVES=4+ALAYA_SPILL_FLAGS=32"
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/base step 600 gpurun_out/r04_helper_base_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000
