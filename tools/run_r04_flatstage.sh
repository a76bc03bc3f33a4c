#!/bin/bash
# GPU-box script (round 4): flat producer staging the next tile before the MFMAs (K <= 128) -- flat parity
# suite, then config 2's shape (and d = 64 / 96) against the saved pre-change build (ab/base).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r04_flatstage_tests.log python -u -m pytest tests/test_flat.py -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/r04_flatstage_tests.log && ! grep -q " failed" gpurun_out/r04_flatstage_tests.log || exit 1
step 300 gpurun_out/r04_flatstage_tree.log python -u tools/ab_flat.py --dims 128,96,64
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/base step 300 gpurun_out/r04_flatstage_base.log python -u tools/ab_flat.py --dims 128,96,64
step 300 gpurun_out/r04_flatstage_tree2.log python -u tools/ab_flat.py --dims 128,96,64
