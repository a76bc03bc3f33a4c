#!/bin/bash
# GPU-box script: device-build tests, then build quality/time at 200k (vs host) and 1M GIST.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_build_tests.log 2>&1 || { tail -40 gpurun_out/gpu_build_tests.log; exit 1; }
tail -3 gpurun_out/gpu_build_tests.log
timeout -k 10 300 python -u tools/build_quality.py --n 200000 --host ${BQ_ARGS} > gpurun_out/bq_200k.jsonl 2> gpurun_out/bq_200k.log || { tail -20 gpurun_out/bq_200k.log; exit 1; }
cat gpurun_out/bq_200k.jsonl
timeout -k 10 400 python -u tools/build_quality.py --n 1000000 --host ${BQ_ARGS} > gpurun_out/bq_1m.jsonl 2> gpurun_out/bq_1m.log || { tail -20 gpurun_out/bq_1m.log; exit 1; }
cat gpurun_out/bq_1m.jsonl
