#!/bin/bash
# GPU-box script (round 4): the whole -m gpu suite, smoke(), then config 5's first-level spill
# threshold sweep on the spill table (1 = the table from the first expansion).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r04_gpu_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/r04_gpu_suite.log && ! grep -q " failed" gpurun_out/r04_gpu_suite.log || exit 1
step 300 gpurun_out/r04_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
step 600 gpurun_out/r04_c5_vislimit.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000 --table 0,-7 --env-sweep ALAYA_VIS_LIMIT=-,1,64
