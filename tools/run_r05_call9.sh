#!/bin/bash
# GPU-box script (round 5, call 9): isolate the helper kernel's cost to its searchers at 1k queries
# (config 5 and SIFT-shaped): helpers unregistered (32), registered but idle (8), polling only (16),
# working (0), and the plain kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/r05_help6_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 1000 --envs="-,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=32,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=8,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=16,ALAYA_HELPERS=1,-"
step 300 gpurun_out/r05_help6_sift.log python -u tools/shape_sweep.py --workload sift --nq 1000 --envs="-,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=32,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=8,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=17,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=1,-"
