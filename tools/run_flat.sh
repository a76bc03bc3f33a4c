#!/bin/bash
# GPU-box script: flat path parity (both contractions), scan diagnostics, config-2 bench in both
# contractions (f32 MFMA via ALAYA_FLAT_F32).  Every GPU step time-limited; stop on error.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flat.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/flat_tests.log 2>&1 || { tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -2 gpurun_out/flat_tests.log
timeout -k 10 300 python -u tools/flat_diag.py > gpurun_out/flat_diag_split.log 2>&1 || { tail -20 gpurun_out/flat_diag_split.log; exit 1; }
ALAYA_FLAT_F32=1 timeout -k 10 300 python -u tools/flat_diag.py > gpurun_out/flat_diag_f32.log 2>&1 || { tail -20 gpurun_out/flat_diag_f32.log; exit 1; }
tail -4 gpurun_out/flat_diag_split.log gpurun_out/flat_diag_f32.log
timeout -k 10 400 python -u bench.py --workload flat --steps 20 --warmup 3 > gpurun_out/bench_flat.json 2> gpurun_out/bench_flat.log || { tail -20 gpurun_out/bench_flat.log; exit 1; }
cat gpurun_out/bench_flat.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flat -o run --output-format csv -- python bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_flat_prof.json 2> gpurun_out/bench_flat_prof.log
