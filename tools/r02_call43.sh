# config 4's batch on one GPU (GIST 1M, 10k queries): PMC traffic at its operating ef, then the bench line with it
source tools/gpu_steps.sh
EF=373 GROUPS_PMC="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" step 1000 gpurun_out/r02_pmc_gist10k.log bash tools/run_pmc.sh gpurun_out/traffic_gist10k.json --nq 10000
cp gpurun_out/traffic_gist10k.json profiles/r02/traffic_gist10k.json
step 900 gpurun_out/r02_gist10k_final.log python -u bench.py --nq 10000 --steps 10 --warmup 2
grep -h '^{' gpurun_out/r02_gist10k_final.log > gpurun_out/r02_gist10k_final.json
