# ring-decoupled flat scan: full GPU suite, config 2 bench (CPU leg), rocprof kernel stats, PMC traffic
source tools/gpu_steps.sh
step 900 gpurun_out/r02_s3_gpu_tests2.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 600 gpurun_out/r02_flat_c2_ring.log python -u bench.py --workload flat --steps 20 --warmup 3
grep -h '^{' gpurun_out/r02_flat_c2_ring.log > gpurun_out/r02_flat_c2_ring.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 300 gpurun_out/r02_flat_c2_ring_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flat_ring -o run -- python bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
step 900 gpurun_out/r02_pmc_flat_ring.log bash tools/run_pmc_flat.sh gpurun_out/traffic_flat_ring.json
