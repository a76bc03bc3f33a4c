# configs 3 and 5 re-run on the final tree so their JSON lines carry the PMC traffic (profiles/r02/traffic_*_c*.json)
source tools/gpu_steps.sh
step 600 gpurun_out/r02_sift_final.log python -u bench.py --workload sift-hnsw --sweep-qps --steps 20 --warmup 3
grep -h '^{' gpurun_out/r02_sift_final.log > gpurun_out/r02_sift_final.json
step 900 gpurun_out/r02_c5_final.log python -u bench.py --workload sq8-ip --steps 20 --warmup 3
grep -h '^{' gpurun_out/r02_c5_final.log > gpurun_out/r02_c5_final.json
