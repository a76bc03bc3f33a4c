#!/bin/bash
# GPU-box script: parity suite on the tree, then tree vs ab/nopre (no second-level visited prefetch)
# on config 5 (spilling queries at 10k), SIFT and GIST.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q " failed" gpurun_out/gpu_suite.log || exit 1
for v in tree nopre; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/sp_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
  step 200 gpurun_out/sp_sift_$v.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000
done
