#!/bin/bash
# GPU-box script (round 4): (1) f32 rows on the spill table -- parity, then config 3 (SIFT 1M, 10k /
# 1k queries) LDS first level vs the spill table at 16 / 20 searchers per CU; (2) the flat scan with
# two consumer waves per producer -- parity (every flat case), then config 2 one vs two consumers.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
source tools/gpu_steps.sh
step 600 gpurun_out/r04_sift_tests.log python -u -m pytest tests/test_visited.py tests/test_flat.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread --maxfail 4
grep -q " passed" gpurun_out/r04_sift_tests.log && ! grep -q " failed" gpurun_out/r04_sift_tests.log || exit 1
step 600 gpurun_out/r04_sift_ab.log python -u tools/shape_sweep.py --workload sift --nq 10000,1000 --max-waves 16,20 --envs="-,ALAYA_SPILL_TABLE_F32=1"
step 300 gpurun_out/r04_flat_ws1.log python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
ALAYA_FLAT_WS2=1 step 300 gpurun_out/r04_flat_ws2.log python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
step 300 gpurun_out/r04_flat_ws1b.log python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
ALAYA_FLAT_WS2=1 step 300 gpurun_out/r04_flat_ws2b.log python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
grep -h '^{' gpurun_out/r04_flat_ws*.log | python -c "import sys, json; [print(json.loads(l)['value'], json.loads(l)['roofline']['kernel_ms']) for l in sys.stdin]"
