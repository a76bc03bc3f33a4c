#!/bin/bash
# GPU-box script: full GPU parity suite, smoke(), config-2 bench with its CPU leg, and the
# rocprofv3 kernel-trace summary of the same flat command.  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py --workload flat --steps 20 --warmup 3 > gpurun_out/bench_flat.json 2> gpurun_out/bench_flat.log || { tail -20 gpurun_out/bench_flat.log; exit 1; }
cat gpurun_out/bench_flat.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flat -o run --output-format csv -- python bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_flat_prof.json 2> gpurun_out/bench_flat_prof.log
