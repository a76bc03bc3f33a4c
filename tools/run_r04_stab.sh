#!/bin/bash
# GPU-box script (round 4): parity of the spill-table second level (forced-spill SQ8 suite, visited
# and SQ8 tests), the torch / engine runtime-order probe, then config 5 at 10k / 1k queries on the
# spill table vs the bitset second level, and table sizes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r04_stab_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_visited.py tests/test_sq8.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread --maxfail 8
grep -q " passed" gpurun_out/r04_stab_tests.log && ! grep -q " failed" gpurun_out/r04_stab_tests.log || exit 1
step 300 gpurun_out/r04_runtime_order.log python -u tools/runtime_order_probe.py
step 900 gpurun_out/r04_stab_c5.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000 --spill-table d,0,13,15
