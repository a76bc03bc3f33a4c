#!/bin/bash
# GPU-box script: the whole -m gpu suite (pass extra pytest args as $@), log under gpurun_out/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 1000 gpurun_out/gpu_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread "$@"
