#!/bin/bash
# GPU-box script mirroring the driver's round end: parity tests, smoke(), default bench (N=1,
# with the CPU leg), then the rocprofv3 kernel-trace summary of the same bench at the chosen ef.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/run_bench_1m.sh || exit $?
cat gpurun_out/bench_1m.json
cut -c1-160 gpurun_out/prof_1m/run_kernel_stats.csv | head -3
