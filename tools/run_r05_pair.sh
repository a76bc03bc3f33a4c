#!/bin/bash
# GPU-box script (round 5): lane loops taken two lanes per trip (ALAYA_PAIR_LOOPS, the tree) against
# one per trip (ab/unpaired): parity tests of the merge / spill-table paths, then SIFT-shaped,
# config 5 and GIST timings on one graph per workload (equal ids hashes = same results).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/r05_pair_tests.log python -u -m pytest tests/test_gpu.py tests/test_sq8_spill.py tests/test_helpers.py tests/test_operating_region.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for v in tree unpaired tree unpaired; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 200 gpurun_out/r05_pair_sift_$v.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --reps 20
done
for v in tree unpaired; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 300 gpurun_out/r05_pair_gist_$v.log python -u tools/shape_sweep.py --workload gist --ef 387 --nq 1000 --reps 20
done
for v in tree unpaired; do
  if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
  step 400 gpurun_out/r05_pair_sq8_$v.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --reps 10
done
