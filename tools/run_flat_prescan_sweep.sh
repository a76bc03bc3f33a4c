cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for S in 0 16 64 128 256; do
ALAYA_FLAT_PRESCAN=$S timeout -k 10 300 python -u bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bf_$S.json 2> gpurun_out/bf_$S.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/bf_$S.json')); print('S=$S', d['value'], d['roofline']['kernel_ms'], d['config']['flagged_queries'])"
done
