#!/bin/bash
# GPU-box script: parity tests, default bench (with CPU leg), then the rocprofv3 kernel-trace
# summary of the same command at the chosen ef.  Every GPU step time-limited; stop on error.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/run_bench_1m.sh || exit $?
cat gpurun_out/bench_1m.json gpurun_out/bench_1m_prof.json
