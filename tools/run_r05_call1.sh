#!/bin/bash
# GPU-box script (round 5, call 1): the forced-spill SQ8 suite with the new prefetch-check kernel,
# then config 5 (10k and 1k queries) on the tree and on the pre-change build (ab/base).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/r05_spill_tests.log python -u -m pytest tests/test_sq8_spill.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
step 600 gpurun_out/r05_c5_tree.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/base step 600 gpurun_out/r05_c5_base.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000
