# final sanity on the committed tree: smoke, default bench, two-rank rehearsal of the shard path (one GPU, gloo)
source tools/gpu_steps.sh
step 300 gpurun_out/r02_end_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step 900 gpurun_out/r02_end_bench.log python -u bench.py
grep -h '^{' gpurun_out/r02_end_bench.log > gpurun_out/r02_end_bench.json
ALAYA_BENCH_REHEARSE=1 step 600 gpurun_out/r02_end_rehearse2.log python -u bench.py --gpus 2 --n 200000 --steps 5 --warmup 1
grep -h '^{' gpurun_out/r02_end_rehearse2.log > gpurun_out/r02_end_rehearse2.json
