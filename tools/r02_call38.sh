# PMC traffic of the search kernel on config 5 (10M x 768 IP SQ8, 1k queries, ef 331)
source tools/gpu_steps.sh
EF=331 GROUPS_PMC="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" step 1100 gpurun_out/r02_pmc_sq8.log bash tools/run_pmc.sh gpurun_out/traffic_sq8_c5.json --workload sq8-ip
