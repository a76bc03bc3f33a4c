#!/bin/bash
# GPU-box script: the whole -m gpu suite, then the default-policy launch sweeps (tools/shape_sweep.py).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 1000 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread
step 600 gpurun_out/sweep_sq8_default.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
step 300 gpurun_out/sweep_sift_default.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000
step 300 gpurun_out/sweep_gist_default.log python -u tools/shape_sweep.py --workload gist --nq 1000,10000
