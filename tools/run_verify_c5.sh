#!/bin/bash
# GPU-box script after a search-kernel change: the parity suite, config 5 at 10k (+ rocprof), then
# the round-end checks (smoke, default bench + rocprof).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread
grep -q " passed" gpurun_out/gpu_suite.log && ! grep -q " failed" gpurun_out/gpu_suite.log || exit 1
bash tools/run_c5_10k.sh || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
bash tools/run_bench_1m.sh
