#!/bin/bash
# GPU-box script: flat parity tests, then config 2 at several smoothing-round thresholds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/flat_tests.log 2>&1 || { tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -1 gpurun_out/flat_tests.log
for S in 32 40 48 64 97 32; do
ALAYA_FLAT_SMOOTH=$S timeout -k 10 300 python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bs_$S.json 2> gpurun_out/bs_$S.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/bs_$S.json')); print('ALAYA_FLAT_SMOOTH=$S', d['value'], d['roofline']['kernel_ms'], d['config']['flagged_queries'])"
done
