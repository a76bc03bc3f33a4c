#!/bin/bash
# GPU-box script: the secondary BASELINE configs with their CPU legs -- config 3 (SIFT-128, 10k
# queries, QPS/recall curve), config 4 on one GPU (GIST 1M, 10k queries), config 5 (10M x 768 IP
# SQ8 + rerank, device-built graph).  Every GPU step time-limited; stop on error.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --workload sift-hnsw --sweep-qps --steps 20 --warmup 3 > gpurun_out/bench_sift.json 2> gpurun_out/bench_sift.log || { tail -20 gpurun_out/bench_sift.log; exit 1; }
timeout -k 10 600 python -u bench.py --nq 10000 --steps 10 --warmup 2 > gpurun_out/bench_gist10k.json 2> gpurun_out/bench_gist10k.log || { tail -20 gpurun_out/bench_gist10k.log; exit 1; }
timeout -k 10 700 python -u bench.py --workload sq8-ip --steps 20 --warmup 3 > gpurun_out/bench_c5_10m.json 2> gpurun_out/bench_c5_10m.log || { tail -20 gpurun_out/bench_c5_10m.log; exit 1; }
python - <<'PY'
import json
for f in ("bench_sift", "bench_gist10k", "bench_c5_10m"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["config"]["ef_search"], d["config"]["recall_at_10"], d["roofline"]["kernel_ms"],
          d["roofline"]["frac"], (d["cpu_baseline"] or {}).get("value"))
PY
