#!/bin/bash
# GPU-box script: flat parity tests + scan diagnostics + config-2 bench (no CPU leg).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/flat_tests.log 2>&1 || { tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -2 gpurun_out/flat_tests.log
timeout -k 10 300 python -u tools/flat_diag.py > gpurun_out/flat_diag_split.log 2>&1 || { tail -20 gpurun_out/flat_diag_split.log; exit 1; }
grep -v amdgpu.ids gpurun_out/flat_diag_split.log | tail -n 6
ALAYA_FLAT_LOCAL_TAU=1 timeout -k 10 300 python -u tools/flat_diag.py > gpurun_out/flat_diag_local.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/flat_diag_local.log | tail -n 6
timeout -k 10 400 python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_flat.json 2> gpurun_out/bench_flat.log || { tail -20 gpurun_out/bench_flat.log; exit 1; }
cat gpurun_out/bench_flat.json
