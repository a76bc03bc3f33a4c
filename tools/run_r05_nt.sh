#!/bin/bash
# GPU-box script (round 5): SQ8 code rows loaded non-temporally (ab/nt) against the tree: the SQ8
# parity suite on the variant, then config 5 at 10k / 1k, alternating, one graph per run.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/nt step 300 gpurun_out/r05_nt_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_sq8.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for v in tree nt tree nt; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/r05_nt_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --reps 10
  cat gpurun_out/r05_nt_sq8_$v.log >> gpurun_out/r05_nt_sq8_all.log
done
