#!/bin/bash
# one GPU call: parity suite on the tree, then tree vs ab/base (descent change)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q " failed" gpurun_out/gpu_suite.log || exit 1
for v in tree base tree base; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 300 gpurun_out/desc_sift_$v.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000
  cat gpurun_out/desc_sift_$v.log >> gpurun_out/desc_sift_all.log
  step 300 gpurun_out/desc_gist_$v.log python -u tools/shape_sweep.py --workload gist --nq 1000
  cat gpurun_out/desc_gist_$v.log >> gpurun_out/desc_gist_all.log
done
