#!/bin/bash
# GPU-box script (round 4): spill-table parity, then config 5 residency / first-level / second-level A/B.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 900 gpurun_out/r04_stab_tests.log python -u -m pytest tests/test_sq8_spill.py tests/test_visited.py tests/test_sq8.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread --maxfail 8
grep -q " passed" gpurun_out/r04_stab_tests.log && ! grep -q " failed" gpurun_out/r04_stab_tests.log || exit 1
step 900 gpurun_out/r04_stab2_c5.log python -u tools/shape_sweep.py --workload sq8 --nq 10000,1000 --spill-table d,0 --max-waves 0,12 --table 0,-8
