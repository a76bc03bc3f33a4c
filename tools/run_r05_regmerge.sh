#!/bin/bash
# GPU-box script (round 5): the register merge for SQ8 pools (ef <= 384, 6 entries per lane; the tree)
# against the LDS merge (ab/ldsmerge): parity tests, then config 5 and SIFT-shaped timings on one
# graph per workload (equal ids hashes = same results).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r05_rm_tests.log python -u -m pytest tests/test_gpu.py tests/test_sq8_spill.py tests/test_helpers.py tests/test_sq8.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for v in tree ldsmerge; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 200 gpurun_out/r05_rm_sift_$v.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --reps 20
done
for v in tree ldsmerge tree ldsmerge; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/r05_rm_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --reps 10
  cat gpurun_out/r05_rm_sq8_$v.log >> gpurun_out/r05_rm_sq8_all.log
done
