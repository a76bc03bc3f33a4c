#!/bin/bash
# GPU-box script (round 5): the full-size parity tests (configs 3, 4, 5 at their bench sizes against
# the restatement), smoke() with the library's build provenance, and a short headline bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 700 gpurun_out/r05_fullsize_tests.log python -u -m pytest tests/test_full_size.py tests/test_abi.py -m "gpu or not gpu" -v -p no:cacheprovider --timeout 400 --timeout-method thread
step 300 gpurun_out/r05_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
