# residency floor: GPU suite on the new build, then config 5 at its full batch (10k queries) with the CPU leg
source tools/gpu_steps.sh
step 900 gpurun_out/r02_floor_gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 1000 gpurun_out/r02_c5_10k_floor.log python -u bench.py --workload sq8-ip --nq 10000 --steps 10 --warmup 2
grep -h '^{' gpurun_out/r02_c5_10k_floor.log > gpurun_out/r02_c5_10k_floor.json
