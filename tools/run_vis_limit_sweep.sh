#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 200 gpurun_out/lim_sift_def.log python -u tools/shape_sweep.py --workload sift --nq 10000 --max-waves 16,20
for pct in 80 90 95; do
  ALAYA_VIS_LIMIT_PCT=$pct step 200 gpurun_out/lim_sift_$pct.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --max-waves 16,20
done
step 400 gpurun_out/lim_sq8_def.log python -u tools/shape_sweep.py --workload sq8 --nq 10000
ALAYA_VIS_LIMIT_PCT=90 step 400 gpurun_out/lim_sq8_90.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000
