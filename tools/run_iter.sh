#!/bin/bash
# GPU-box script for one optimisation iteration: HBM probe, flat diag + flat tests, search parity,
# 1M bench (no CPU leg) and the phase profile.  Every GPU step has its own time limit; stop on error.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 tools/hbm_probe > gpurun_out/hbm_probe.log 2>&1 || exit $?
timeout -k 10 300 python tools/flat_diag.py > gpurun_out/flat_diag.log 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 900 python bench.py --steps 20 --warmup 3 --ef 400 --no-cpu-baseline > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.log || exit $?
timeout -k 10 600 python tools/profile_phases.py --ef 400 > gpurun_out/phases.log 2>&1 || exit $?
