#!/bin/bash
# GPU-box script (round 4): row warm-up A/B (ALAYA_SPILL_FLAGS=8 turns it on) on SIFT and GIST shapes,
# plus the parity tests of the small-row kernels with it on.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
ALAYA_SPILL_FLAGS=8 step 400 gpurun_out/r04_warm_tests.log python -u -m pytest tests/test_gpu.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "c1 or ties or shapes"
step 400 gpurun_out/r04_warm_sift.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --env-sweep ALAYA_SPILL_FLAGS=-,8,-,8
