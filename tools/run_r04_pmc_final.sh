#!/bin/bash
# GPU-box script (round 4, final tree): PMC traffic of the search kernel at the headline's operating
# point (GIST 1M / 1k, ef 387) and config 3's (SIFT-shaped 1M / 10k, ef 70).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
EF=387 bash tools/run_pmc.sh gpurun_out/traffic.json || exit $?
EF=70 bash tools/run_pmc.sh gpurun_out/traffic_sift_c3.json --workload sift-hnsw || exit $?
