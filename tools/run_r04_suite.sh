#!/bin/bash
# GPU-box script (round 4): the whole -m gpu suite, smoke(), and config 5 at 10k / 1k queries.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 1100 gpurun_out/r04_gpu_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/r04_gpu_suite.log && ! grep -q " failed" gpurun_out/r04_gpu_suite.log || exit 1
step 300 gpurun_out/r04_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
