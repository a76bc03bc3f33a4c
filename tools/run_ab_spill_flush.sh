#!/bin/bash
# GPU-box script: parity suite on the tree, then tree vs ab/noflush (first level kept as a lookup
# after a spill) on config 5 at 10k / 1k queries.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q " failed" gpurun_out/gpu_suite.log || exit 1
for v in tree noflush; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/fl_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
  cat gpurun_out/fl_sq8_$v.log >> gpurun_out/fl_sq8_all.log
done
