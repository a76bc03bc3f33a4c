#!/bin/bash
# GPU-box script: launch-shape sweeps (tools/shape_sweep.py) for config 5 (SQ8 10M), config 3
# (SIFT 1M) and config 4 / the metric (GIST 1M), each step time-limited; logs under gpurun_out/.
# AB_DIRS: saved package builds (ab/<name>) swept too, for A/B across kernel variants.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
for v in tree ${AB_DIRS}; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  if [ -n "$SQ8" ]; then step 700 gpurun_out/sweep_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --nq ${SQ8_NQ:-10000,1000} --waves ${SQ8_WAVES:-0} --table=${SQ8_TABLE:-0}; fi
  if [ -n "$SIFT" ]; then step 400 gpurun_out/sweep_sift_$v.log python -u tools/shape_sweep.py --workload sift --nq ${SIFT_NQ:-10000,1000} --waves ${SIFT_WAVES:-0} --table=${SIFT_TABLE:-0}; fi
  if [ -n "$GIST" ]; then step 400 gpurun_out/sweep_gist_$v.log python -u tools/shape_sweep.py --workload gist --nq ${GIST_NQ:-1000} --waves ${GIST_WAVES:-0} --table=${GIST_TABLE:-0}; fi
done
