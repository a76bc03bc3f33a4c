#!/bin/bash
# GPU-box script (round 5): query order and cache locality -- the same batch in batch order, grouped by
# nearest pivot row with group x on the first round's XCD x, and grouped contiguously; ids compared in
# batch order.  Config 5, SIFT-shaped and GIST-shaped.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 500 gpurun_out/r05_order_sq8.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 10000,1000 --reps 10 --order batch,xcd,sorted,batch,xcd,sorted
step 200 gpurun_out/r05_order_sift.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --reps 20 --order batch,xcd,sorted,batch,xcd,sorted
step 300 gpurun_out/r05_order_gist.log python -u tools/shape_sweep.py --workload gist --ef 387 --nq 1000,10000 --reps 10 --order batch,xcd,sorted,batch
