#!/bin/bash
# GPU-box script (round 5, call 5): helpers v3 (searcher-side state in registers, pool_pop reports
# the next two entries, helper back-off) -- parity, coverage, stamped phases.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_helpers_tests.log python -u -m pytest tests/test_helpers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r05_helpers_tests.log && ! grep -q -E " failed| error" gpurun_out/r05_helpers_tests.log || exit 1
step 300 gpurun_out/r05_help4_sift.log python -u tools/shape_sweep.py --workload sift --nq 1000,10000 --envs="-,ALAYA_HELPERS=1,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=2"
ALAYA_HELPERS=1 step 300 gpurun_out/r05_phases_sift1k_help.log python -u tools/profile_phases.py --workload sift --builder gpu --nq 1000 --ef 70
step 600 gpurun_out/r05_help4_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 1000,10000 --envs="-,ALAYA_HELPERS=1"
ALAYA_HELPERS=1 step 400 gpurun_out/r05_phases_c5_1k_help.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 1000 --ef 368
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/wgscope step 600 gpurun_out/r05_c5_wgscope.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000
