#!/bin/bash
# GPU-box script (round 5, call 8): where the searchers' time goes with helpers -- helpers that leave
# at once (bookkeeping only) or only poll, stamped phases; the two-waves wide-row kernel's parity and
# the automatic policy around 1,024 GIST-shaped queries.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 300 gpurun_out/r05_two_waves_tests.log python -u -m pytest tests/test_gpu.py -k "two_waves or gist_shaped" -q -p no:cacheprovider --timeout 120 --timeout-method thread
for f in 8 16; do
  ALAYA_HELPERS=1 ALAYA_HELP_FLAGS=$f step 400 gpurun_out/r05_phases_c5_1k_flags$f.log python -u tools/profile_phases.py --workload sq8 --n 10000000 --nq 1000 --ef 368
done
step 600 gpurun_out/r05_gist_two_waves.log python -u tools/shape_sweep.py --workload gist --ef 373 --nq 1000,1250,1536,1792,2048 --envs="-,ALAYA_TWO_WAVES=0,ALAYA_TWO_WAVES=1"
