#!/bin/bash
# GPU-box script (round 5, call 7): helpers at depth 1 (the tree) and 2 (ab/depth2), visited hint on
# (default) / off (ALAYA_HELP_FLAGS=1), with the helpers' row counts -- SIFT-shaped and config 5.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_helpers_tests.log python -u -m pytest tests/test_helpers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r05_helpers_tests.log && ! grep -q -E " failed| error" gpurun_out/r05_helpers_tests.log || exit 1
step 300 gpurun_out/r05_help5_sift.log python -u tools/shape_sweep.py --workload sift --nq 1000,10000 --envs="-,ALAYA_HELPERS=1,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=1"
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/depth2 step 300 gpurun_out/r05_help5_sift_d2.log python -u tools/shape_sweep.py --workload sift --nq 1000,10000 --envs="ALAYA_HELPERS=1"
step 600 gpurun_out/r05_help5_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 1000,10000 --envs="-,ALAYA_HELPERS=1,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=1"
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/depth2 step 600 gpurun_out/r05_help5_c5_d2.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 1000,10000 --envs="ALAYA_HELPERS=1"
ALAYA_HELPERS=1 step 400 gpurun_out/r05_phases_c5_1k_help_d1.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 1000 --ef 368
