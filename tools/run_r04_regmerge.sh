#!/bin/bash
# GPU-box script (round 4): register merge for ef <= 128 pools -- test_gpu.py parity (ties included),
# SIFT A/B against the saved pre-change build (ab/base), then the round-end run (tools/run_final.sh).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r04_regmerge_tests.log python -u -m pytest tests/test_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r04_regmerge_tests.log && ! grep -q " failed" gpurun_out/r04_regmerge_tests.log || exit 1
AB="base" bash tools/run_ab_sift.sh || exit $?
bash tools/run_final.sh
