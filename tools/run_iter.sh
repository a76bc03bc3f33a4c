#!/bin/bash
# GPU-box script for one optimisation iteration: parity tests, SIFT phase profile, fixed-ef benches
# (SIFT config 3 at ef 85, GIST at ef 400, SQ8 1M at ef 175) on device-built graphs (deterministic, so
# runs compare).  Every GPU step time-limited.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u tools/profile_phases.py --workload sift --nq 10000 --ef 85 > gpurun_out/phases_sift.log 2>&1 || exit $?
grep -E "expansion|prefetch" gpurun_out/phases_sift.log
timeout -k 10 300 python -u bench.py --workload sift-hnsw --builder gpu --ef 85 --no-cpu-baseline > gpurun_out/b_sift.json 2> gpurun_out/b_sift.log || exit $?
timeout -k 10 400 python -u bench.py --builder gpu --ef 400 --no-cpu-baseline > gpurun_out/b_gist.json 2> gpurun_out/b_gist.log || exit $?
timeout -k 10 300 python -u bench.py --workload sq8-ip --n 1000000 --builder gpu --ef 175 --no-cpu-baseline > gpurun_out/b_sq8.json 2> gpurun_out/b_sq8.log || exit $?
python - <<'PY'
import json
for f in ("b_sift", "b_gist", "b_sq8"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["config"]["ef_search"], d["config"]["recall_at_10"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
PY
