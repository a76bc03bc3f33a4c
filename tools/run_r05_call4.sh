#!/bin/bash
# GPU-box script (round 5, call 4): helpers v2 diagnostics -- memo coverage per expansion and the
# stamped phase split with and without helpers (SIFT-shaped 1M, config 5 10M), 1k queries.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_helpers_tests.log python -u -m pytest tests/test_helpers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r05_helpers_tests.log && ! grep -q -E " failed| error" gpurun_out/r05_helpers_tests.log || exit 1
step 300 gpurun_out/r05_help3_sift.log python -u tools/shape_sweep.py --workload sift --nq 1000,10000 --envs="-,ALAYA_HELPERS=1,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=2"
step 300 gpurun_out/r05_phases_sift1k.log python -u tools/profile_phases.py --workload sift --builder gpu --nq 1000 --ef 70
ALAYA_HELPERS=1 step 300 gpurun_out/r05_phases_sift1k_help.log python -u tools/profile_phases.py --workload sift --builder gpu --nq 1000 --ef 70
step 400 gpurun_out/r05_phases_c5_1k.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 1000 --ef 368
ALAYA_HELPERS=1 step 400 gpurun_out/r05_phases_c5_1k_help.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 1000 --ef 368
