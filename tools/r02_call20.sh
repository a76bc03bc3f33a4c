# flat config 2 on the warp-specialised scan: PMC traffic passes (-> profiles/r02/traffic_flat.json),
# then the bench line with its CPU leg and a rocprofv3 kernel-stats summary of the same command
source tools/gpu_steps.sh
step 900 gpurun_out/r02_pmc_flat.log bash tools/run_pmc_flat.sh gpurun_out/traffic_flat.json
step 400 gpurun_out/r02_flat_c2_final.log python -u bench.py --workload flat --steps 20 --warmup 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 300 gpurun_out/r02_flat_c2_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flat_c2 -o run -- python bench.py --workload flat --steps 20 --warmup 3 --no-cpu-baseline
