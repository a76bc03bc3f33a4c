#!/bin/bash
# GPU-box script (round 4): tail helpers reading the sibling's pool (2nd-4th unchecked entries)
# -- parity with helpers on, then config 5 A/B (ALAYA_SPILL_FLAGS=32) and the committed build.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
ALAYA_SPILL_FLAGS=32 step 400 gpurun_out/r04_helper2_tests.log python -u -m pytest tests/test_sq8.py tests/test_sq8_spill.py tests/test_visited.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r04_helper2_tests.log && ! grep -q " failed" gpurun_out/r04_helper2_tests.log || exit 1
step 600 gpurun_out/r04_helper2_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --envs="-,ALAYA_SPILL_FLAGS=32,-,ALAYA_SPILL_FLAGS=32"
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/base step 600 gpurun_out/r04_helper2_base_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000
