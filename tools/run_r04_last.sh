#!/bin/bash
# GPU-box script (round 4, last): the driver's round-end commands on the final tree -- the -m gpu
# suite, smoke(), and bench.py with its defaults.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/last_suite.log python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/last_suite.log && ! grep -q " failed" gpurun_out/last_suite.log || exit 1
step 300 gpurun_out/last_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
step 600 gpurun_out/last_bench.log python -u bench.py
grep '^{' gpurun_out/last_bench.log > gpurun_out/last_bench.json
