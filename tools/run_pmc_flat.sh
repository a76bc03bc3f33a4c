#!/bin/bash
# PMC passes for the flat scan kernel (flat_scan_kernel / flat_scan_ws_kernel / flat_scan_wide_kernel /
# flat_scan_tiles_kernel, whichever the dispatch picks; the single-role scan's prescan launch -- the
# same template with kMin = true -- is excluded) on one flat workload (one counter group per pass,
# kernel-trace only),
# summarised into $1 (default gpurun_out/traffic_flat.json; bench.py reads profiles/r*/traffic_flat*.json).
# Extra arguments go to bench.py (e.g. --dim 960).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${1:-gpurun_out/traffic_flat.json}
shift
ARGS="--workload flat --steps 5 --warmup 1 --no-cpu-baseline $*"
rm -rf gpurun_out/pmcf_*
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex flat_scan_ --kernel-exclude-regex 'tiles_kernel<[0-9]+, true>' --output-format csv -d gpurun_out/pmcf_$name -o run -- python bench.py $ARGS > gpurun_out/pmcf_$name.json 2> gpurun_out/pmcf_$name.log || exit $?
done
python tools/pmc_summary.py gpurun_out $OUT flat > /dev/null || exit $?
rm -f gpurun_out/pmcf_*/run_kernel_trace.csv
python -c "import json, sys; t=json.load(open(sys.argv[1])); print(t['kernel'], t['hbm_read_bytes_per_launch'], t['traffic_over_algorithmic'], t['l2_hit_rate'])" $OUT
