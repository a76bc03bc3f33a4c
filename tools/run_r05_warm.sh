#!/bin/bash
# GPU-box script (round 5): the LDS-DMA row warm-up of spilled SQ8 queries (the tree) against no
# warm-up (ab/nowarm): SQ8 parity suites on the tree, then config 5 at 10k / 1k with helpers on
# (default) and off, one graph per run.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r05_warm_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_sq8.py tests/test_helpers.py tests/test_visited.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for v in tree nowarm tree nowarm; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/r05_warm_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --reps 10 --envs="-,ALAYA_HELPERS=0"
  cat gpurun_out/r05_warm_sq8_$v.log >> gpurun_out/r05_warm_sq8_all.log
done
