#!/bin/bash
# GPU-box script: device-build tests, then build quality/time at 1M GIST (vs host), then a
# rocprofv3 kernel-trace summary of a device-only 1M build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_build.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_build_tests.log 2>&1 || { tail -40 gpurun_out/gpu_build_tests.log; exit 1; }
tail -3 gpurun_out/gpu_build_tests.log
timeout -k 10 400 python -u tools/build_quality.py --n 1000000 ${BQ_HOST---host} ${BQ_ARGS} > gpurun_out/bq_1m.jsonl 2> gpurun_out/bq_1m.log || { tail -20 gpurun_out/bq_1m.log; exit 1; }
cat gpurun_out/bq_1m.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_build -o run --output-format csv -- python -u tools/build_quality.py --n 1000000 --efs 400 ${BQ_ARGS} > gpurun_out/bq_1m_prof.jsonl 2> gpurun_out/bq_1m_prof.log || { tail -20 gpurun_out/bq_1m_prof.log; exit 1; }
cut -c1-220 gpurun_out/prof_build/run_kernel_stats.csv | head -14
