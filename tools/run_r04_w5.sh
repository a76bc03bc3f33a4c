#!/bin/bash
# GPU-box script (round 4): config 5 with the SQ8 kernel held to 5 waves per SIMD (96 VGPRs, scratch
# in the loop) and 20 searchers per CU, against the tree (4 waves, 16 per CU).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 500 gpurun_out/r04_w5_tree.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000
for v in w5dw24 w5; do
  ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v step 500 gpurun_out/r04_w5_$v.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --max-waves 16,20
done
