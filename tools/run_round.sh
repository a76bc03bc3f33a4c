#!/bin/bash
# GPU-box script: parity tests, 1M bench (+counters), phase profile.  Each GPU step time-limited.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.log || exit $?
cat gpurun_out/bench_1m.json
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 python tools/profile_phases.py --ef ${PROFILE_EF:-400} > gpurun_out/phases.log 2>&1 || exit $?
  cat gpurun_out/phases.log
fi
