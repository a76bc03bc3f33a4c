#!/bin/bash
# GPU-box script: the parity suite against the self-contained flush copy (ab/flush), then config 5
# sweeps of the tree and of the copy (equal ids hashes = same results).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
( cd ab/flush && step 600 ../../gpurun_out/flush_suite.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread )
grep -q " passed" gpurun_out/flush_suite.log && ! grep -q " failed" gpurun_out/flush_suite.log || exit 1
grep -q "ab/flush" gpurun_out/flush_suite.log; true
step 400 gpurun_out/fl_sq8_tree.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/flush
step 400 gpurun_out/fl_sq8_flush.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
