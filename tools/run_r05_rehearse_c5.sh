#!/bin/bash
# GPU-box script (round 5): the config-4 1,250-query full-size parity case, config 3's PMC traffic
# at ef 70, then config 5's N = 8 layouts rehearsed on one MI355X with the round-5 kernels.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_fullsize_c4.log python -u -m pytest tests/test_full_size.py -m gpu -v -k "config4" -p no:cacheprovider --timeout 250 --timeout-method thread
EF=70 bash tools/run_pmc.sh gpurun_out/traffic_sift_c3.json --workload sift-hnsw || exit $?
step 900 gpurun_out/r05_rehearsal_c5.log python -u tools/shard_rehearsal.py --workload sq8 --nq 10000 --out gpurun_out/shard_rehearsal_c5_10k.json
