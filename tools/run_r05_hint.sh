#!/bin/bash
# GPU-box script (round 5): the helper tests after the sibling-table hint reads became relaxed atomics,
# then config 5 at 1k / 10k with and without helpers (same graph, ids hashes compared).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r05_hint_tests.log python -u -m pytest tests/test_helpers.py tests/test_sq8_spill.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
step 600 gpurun_out/r05_hint_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 1000,10000 --envs="ALAYA_HELPERS=0,-,ALAYA_HELPERS=0,-" --reps 10
