#!/bin/bash
# one GPU call: SIFT 10k visited-table layouts / sizes at the default residency, SQ counters of
# config 5 at 10k queries (tools/run_pmc_sq.sh)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/sw_sift_visited.log python -u tools/shape_sweep.py --workload sift --nq 10000 --visited 0,1,2 --table 0,-11,-13
WORKLOAD=sq8 NQ=10000 EF=340 bash tools/run_pmc_sq.sh
