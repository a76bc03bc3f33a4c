#!/bin/bash
# GPU-box script (round 5): config 5 with the plain SQ8 kernel's register merge (ab/regplain) against
# the tree, helpers on (default) and off, 10k / 1k queries, one graph per run.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/regplain
step 300 gpurun_out/r05_rp_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_sq8.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for v in tree regplain tree regplain; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/r05_rp_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --reps 10 --envs="-,ALAYA_HELPERS=0"
  cat gpurun_out/r05_rp_sq8_$v.log >> gpurun_out/r05_rp_sq8_all.log
done
