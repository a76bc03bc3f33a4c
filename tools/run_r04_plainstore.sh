#!/bin/bash
# GPU-box script (round 4): spill-table entries and clears as plain stores (ALAYA_SPILL_FLAGS=16:
# the lines stay in the XCD's L2) against agent-scope stores (sc1: each 16-bit store a fabric write
# that drops the line) -- parity of the spilled SQ8 paths with the flag, then config 5 at 10k / 1k.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
ALAYA_SPILL_FLAGS=16 step 500 gpurun_out/r04_plain_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_visited.py tests/test_sq8.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r04_plain_tests.log && ! grep -q " failed" gpurun_out/r04_plain_tests.log || exit 1
step 900 gpurun_out/r04_plain_c5.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000 --envs="-,ALAYA_SPILL_FLAGS=16,-,ALAYA_SPILL_FLAGS=16"
