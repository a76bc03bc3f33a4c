#!/bin/bash
# GPU-box script: A/B of the search kernels, current tree vs ab_old/ (a build of the tree before
# the row_distances split), on deterministic device-built graphs, interleaved new/old/new/old.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/time_fixed.py > gpurun_out/ab_new1.log 2>&1 || { tail gpurun_out/ab_new1.log; exit 1; }
(cd ab_old && timeout -k 10 300 python -u tools/time_fixed.py) > gpurun_out/ab_old1.log 2>&1 || { tail gpurun_out/ab_old1.log; exit 1; }
timeout -k 10 300 python -u tools/time_fixed.py > gpurun_out/ab_new2.log 2>&1 || { tail gpurun_out/ab_new2.log; exit 1; }
(cd ab_old && timeout -k 10 300 python -u tools/time_fixed.py) > gpurun_out/ab_old2.log 2>&1 || { tail gpurun_out/ab_old2.log; exit 1; }
for f in ab_new1 ab_old1 ab_new2 ab_old2; do echo "== $f"; grep "ms" gpurun_out/$f.log; done
