#!/bin/bash
# GPU-box script: launch-shape A/B of the tree against saved variant builds (ab/<name>) on one
# device-built graph per run (equal ids hashes = same results).
# usage: AB="name1 name2" [W=sift] [NQ=10000,1000] [EF=70] bash tools/run_ab_sift.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
W=${W:-sift}
for v in tree ${AB}; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  EFARG=""
  if [ -n "$EF" ]; then EFARG="--ef $EF"; fi
  step 400 gpurun_out/ab_${W}_$v.log python -u tools/shape_sweep.py --workload $W --nq ${NQ:-10000,1000} $EFARG
done
