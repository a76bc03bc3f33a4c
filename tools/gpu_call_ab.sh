#!/bin/bash
# one GPU call: per-phase stamps at 10k queries (config 5 and SIFT), plain and fine-stamped builds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 400 gpurun_out/ph_sq8_10k.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 10000 --ef 340
step 200 gpurun_out/ph_sift_10k.log python -u tools/profile_phases.py --workload sift --n 1000000 --nq 10000 --ef 70 --builder gpu
export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/fine
step 400 gpurun_out/ph_sq8_10k_fine.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 10000 --ef 340 --fine
step 200 gpurun_out/ph_sift_10k_fine.log python -u tools/profile_phases.py --workload sift --n 1000000 --nq 10000 --ef 70 --builder gpu --fine
