cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --steps 20 --warmup 3 --dump-counters gpurun_out/counters_1m.npy > gpurun_out/bench_1m.json 2> gpurun_out/bench_1m.log || exit $?
EF=$(python -c "import json;print(json.load(open('gpurun_out/bench_1m.json'))['config']['ef_search'])")
echo "ef=$EF" >> gpurun_out/bench_1m.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_1m -o run --output-format csv -- python bench.py --ef $EF --steps 20 --warmup 3 --no-cpu-baseline --no-tail-probe > gpurun_out/bench_1m_prof.json 2> gpurun_out/bench_1m_prof.log
