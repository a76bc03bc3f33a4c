#!/bin/bash
# GPU-box script: the config-3 (SIFT-128, 10k queries, QPS/recall curve) and config-5-shape (768-d IP
# SQ8 + rerank) bench legs, then the default GIST bench.  Every GPU step time-limited; stop on error.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --workload sift-hnsw --sweep-qps --steps 20 --warmup 3 > gpurun_out/bench_sift.json 2> gpurun_out/bench_sift.log || exit $?
timeout -k 10 500 python bench.py --workload sq8-ip --steps 20 --warmup 3 > gpurun_out/bench_sq8ip.json 2> gpurun_out/bench_sq8ip.log || exit $?
