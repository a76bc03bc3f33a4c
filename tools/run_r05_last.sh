#!/bin/bash
# GPU-box script (round 5, last): smoke() and the core parity tests on the tree as committed.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_last_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
step 400 gpurun_out/r05_last_tests.log python -u -m pytest tests/test_abi.py tests/test_gpu.py tests/test_helpers.py tests/test_sq8_spill.py -m "gpu or not gpu" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
