# config 5 at its full query count (10k queries on one GPU), CPU leg included
source tools/gpu_steps.sh
step 1100 gpurun_out/r02_c5_10k.log python -u bench.py --workload sq8-ip --nq 10000 --steps 10 --warmup 2
grep -h '^{' gpurun_out/r02_c5_10k.log > gpurun_out/r02_c5_10k.json
