#!/bin/bash
# PMC passes for the search kernel at the bench operating point (one counter group per pass,
# kernel-trace only, as MI355X_MICROARCH.md's rocprofv3 section prescribes), then the traffic
# summary bench.py reports as roofline.traffic.  Device-built graph (deterministic, 8 s build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
EF=${EF:-400}
ARGS="--ef $EF --steps 5 --warmup 1 --no-cpu-baseline --builder gpu"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  name=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex hnsw_search_kernel --output-format csv -d gpurun_out/pmc_$name -o run -- python bench.py $ARGS > gpurun_out/pmc_$name.json 2> gpurun_out/pmc_$name.log || exit $?
done
python tools/pmc_summary.py gpurun_out gpurun_out/traffic.json > /dev/null || exit $?
rm -f gpurun_out/pmc_*/run_kernel_trace.csv
du -sh gpurun_out
echo pmc done
python -c "import json; t=json.load(open('gpurun_out/traffic.json')); print(t['traffic_over_algorithmic'], t['l2_hit_rate'], t['rdreq_x64_over_fetch'], t['profiled_kernel_ms'])"
