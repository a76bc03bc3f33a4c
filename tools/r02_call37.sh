# PMC traffic of the search kernel on config 3 (SIFT 1M, 10k queries, ef 70)
source tools/gpu_steps.sh
EF=70 step 1100 gpurun_out/r02_pmc_sift.log bash tools/run_pmc.sh gpurun_out/traffic_sift_c3.json --workload sift-hnsw
