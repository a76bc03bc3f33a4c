#!/bin/bash
# GPU-box script (round 5, call 10): helpers with relaxed publishing (SIFT-shaped and config 5, 1k /
# 10k), then config 2 (flat) on the current scan -- bench with its CPU leg, rocprofv3 kernel-trace
# summary of the same command, PMC traffic passes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_helpers_tests.log python -u -m pytest tests/test_helpers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r05_helpers_tests.log && ! grep -q -E " failed| error" gpurun_out/r05_helpers_tests.log || exit 1
step 300 gpurun_out/r05_help7_sift.log python -u tools/shape_sweep.py --workload sift --nq 1000,10000 --envs="-,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=8,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=1,ALAYA_HELPERS=1"
step 600 gpurun_out/r05_help7_c5.log python -u tools/shape_sweep.py --workload sq8 --ef 368 --nq 1000,10000 --envs="-,ALAYA_HELPERS=1+ALAYA_HELP_FLAGS=8,ALAYA_HELPERS=1,-,ALAYA_HELPERS=1"
step 400 gpurun_out/r05_flat_bench.log python -u bench.py --workload flat --steps 20 --warmup 3
grep '^{' gpurun_out/r05_flat_bench.log > gpurun_out/r05_flat_bench.json
step 300 gpurun_out/r05_flat_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r05_prof_flat -o run --output-format csv -- python bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
step 600 gpurun_out/r05_flat_pmc.log bash tools/run_pmc_flat.sh gpurun_out/r05_traffic_flat.json
