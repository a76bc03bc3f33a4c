#!/bin/bash
# PMC passes for the search kernel at a bench operating point (one counter group per pass,
# kernel-trace only, as MI355X_MICROARCH.md's rocprofv3 section prescribes), then the traffic
# summary bench.py reports as roofline.traffic.  Device-built graph (deterministic).
# usage: tools/run_pmc.sh [OUT (default gpurun_out/traffic.json)] [extra bench.py args, e.g. --workload sift-hnsw]
# EF (default 400) fixes the operating point; GROUPS overrides the counter groups.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${1:-gpurun_out/traffic.json}
shift
EF=${EF:-400}
ARGS="--ef $EF --steps 5 --warmup 1 --no-cpu-baseline --no-tail-probe --builder gpu $*"
rm -rf gpurun_out/pmc_*
IFS=';' read -ra PASSES <<< "${GROUPS_PMC:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum}"
for grp in "${PASSES[@]}"; do
  name=$(echo $grp | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex hnsw_search_kernel --output-format csv -d gpurun_out/pmc_$name -o run -- python bench.py $ARGS > gpurun_out/pmc_$name.json 2> gpurun_out/pmc_$name.log || exit $?
done
python tools/pmc_summary.py gpurun_out $OUT > /dev/null || exit $?
rm -f gpurun_out/pmc_*/run_kernel_trace.csv
du -sh gpurun_out
echo pmc done
python -c "import json, sys; t=json.load(open(sys.argv[1])); print(t['traffic_over_algorithmic'], t['l2_hit_rate'], t['rdreq_x64_over_fetch'], t['profiled_kernel_ms'])" $OUT
