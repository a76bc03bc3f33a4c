#!/bin/bash
# GPU-box script (round 4): PMC traffic of config 5's search kernel at its 10k-query operating point
# (spill table), one counter group per pass (tools/run_pmc.sh).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EF=368 bash tools/run_pmc.sh gpurun_out/traffic_sq8_c5_10k.json --workload sq8-ip --nq 10000
