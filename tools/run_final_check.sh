#!/bin/bash
# GPU-box script: the round-end checks on the final tree -- GPU parity suite and smoke().
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_flat.json 2> gpurun_out/bench_flat.log || { tail -20 gpurun_out/bench_flat.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_flat.json')); print('flat', d['value'], d['roofline']['kernel_ms'], d['config']['flagged_queries'])"
