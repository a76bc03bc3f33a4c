#!/bin/bash
# GPU-box script: default-policy sweeps of the tree and of saved variant builds (ab/<name>).
# usage: AB_SQ8="names" AB_SIFT="names" bash tools/run_ab_sweeps.sh   (tree always included)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
for v in tree ${AB_SQ8}; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 600 gpurun_out/ab_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000 --table=${SQ8_TABLE:-0}
done
for v in tree ${AB_SIFT}; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 300 gpurun_out/ab_sift_$v.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --table=${SIFT_TABLE:-0}
done
if [ -n "$GIST" ]; then unset ALAYA_AB_ROOT; step 300 gpurun_out/ab_gist_tree.log python -u tools/shape_sweep.py --workload gist --nq 1000,10000; fi
