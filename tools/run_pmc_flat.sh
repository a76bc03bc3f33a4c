#!/bin/bash
# PMC passes for the flat scan kernel on config 2 (one counter group per pass, kernel-trace only),
# summarised into gpurun_out/traffic_flat.json (copied to profiles/r01/ for bench.py).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--workload flat --steps 5 --warmup 1 --no-cpu-baseline"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex flat_scan_kernel --output-format csv -d gpurun_out/pmcf_$name -o run -- python bench.py $ARGS > gpurun_out/pmcf_$name.json 2> gpurun_out/pmcf_$name.log || exit $?
done
python tools/pmc_summary.py gpurun_out gpurun_out/traffic_flat.json flat > /dev/null || exit $?
rm -f gpurun_out/pmcf_*/run_kernel_trace.csv
python -c "import json; t=json.load(open('gpurun_out/traffic_flat.json')); print(t['hbm_read_bytes_per_launch'], t['traffic_over_algorithmic'], t['l2_hit_rate'])"
