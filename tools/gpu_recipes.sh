#!/bin/bash
# GPU-box driver (round 6): one parameterised entry point for the GPU runs this repo makes, instead
# of a one-off script per call.  Every GPU step runs under its own time limit (tools/gpu_steps.sh);
# logs and JSON lines go to gpurun_out/<prefix>_*.  Run from the repo root under gpurun:
#   gpurun --timeout 1200 -- bash tools/gpu_recipes.sh <recipe> [prefix]
# Recipes:
#   suite       the whole -m gpu suite, then smoke()
#   headline    the default bench (GIST 1M / 1k, CPU leg) + its rocprofv3 kernel summary at the chosen ef
#   c3 | c4 | c5 | flat
#               the secondary configs (SIFT-shaped 1M / 10k; GIST 1M / 10k; 10M x 768 IP SQ8 + rerank /
#               10k; flat 1M x 128 / 1k), each with its CPU leg and a rocprofv3 summary of the same command
#   pmc-c4 | pmc-c5 | pmc-flat
#               HBM traffic (PMC passes, tools/run_pmc.sh / run_pmc_flat.sh) at the config's operating point
#   rehearse8   the driver's N = 8 command at its defaults (config 4) with every rank on cuda:0 over gloo
#   rehearse8-sq8
#               N = 8 on the config-5 workload at N8_ROWS rows (default 4M) and N8_NQ queries (default 10k), every rank on cuda:0
#   shard-rehearsal <gist|sq8>
#               tools/shard_rehearsal.py at config 4's / config 5's batch: every layout's shard graphs
#               built and timed on one GPU, the predicted N = 8 efficiencies
#   build-quality
#               the device HNSW build's tests, recall of the device graph vs the host builder at 1M
#               (tools/build_quality.py) and a rocprofv3 summary of the build kernels
#   graph-quality
#               the device-built graph's recall@10-vs-ef curve on the headline data (tools/graph_quality.py;
#               its host single-thread counterpart runs on the CPU)
#   ab-flat "v1 v2 ..."
#               config 2's flat scan timed per variant (tools/ab_flat.py; "tree" = this tree's build,
#               anything else = a saved build ab/<name>, tools/build_ab.sh), interleaved twice
#   ab-search <sift|sq8|gist> "v1 v2 ..." [shape_sweep args]
#               the graph search per variant on one device-built graph per run (tools/shape_sweep.py),
#               interleaved twice; equal ids hashes = identical results
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
source tools/gpu_steps.sh
recipe=$1
P=${2:-r06}
json() { grep '^{' "$1" > "${1%.log}.json" || true; }
prof() {  # prof <limit> <name> <bench args...>: rocprofv3 kernel-trace summary of a bench command
  local secs=$1 name=$2
  shift 2
  step "$secs" gpurun_out/${P}_${name}_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_${name} -o run \
    --output-format csv -- python -u bench.py "$@" --no-cpu-baseline --no-tail-probe
  find gpurun_out/prof_${P}_${name} -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${P}_${name}_kernel_stats.csv
  rm -rf gpurun_out/prof_${P}_${name}
}
ef_of() { python -c "import json,sys;print(json.load(open(sys.argv[1]))['config']['ef_search'])" "$1"; }
case "$recipe" in
  suite)
    step 1000 gpurun_out/${P}_suite.log python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
    step 300 gpurun_out/${P}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
    ;;
  headline)
    step 600 gpurun_out/${P}_headline.log python -u bench.py
    json gpurun_out/${P}_headline.log
    prof 400 headline --ef "$(ef_of gpurun_out/${P}_headline.json)"
    ;;
  c3)
    step 600 gpurun_out/${P}_c3.log python -u bench.py --workload sift-hnsw --nq 10000
    json gpurun_out/${P}_c3.log
    prof 400 c3 --workload sift-hnsw --nq 10000 --ef "$(ef_of gpurun_out/${P}_c3.json)"
    ;;
  c4)
    step 900 gpurun_out/${P}_c4.log python -u bench.py --nq 10000
    json gpurun_out/${P}_c4.log
    prof 600 c4 --nq 10000 --ef "$(ef_of gpurun_out/${P}_c4.json)"
    ;;
  c5)
    step 1000 gpurun_out/${P}_c5.log python -u bench.py --workload sq8-ip --nq 10000
    json gpurun_out/${P}_c5.log
    prof 900 c5 --workload sq8-ip --nq 10000 --ef "$(ef_of gpurun_out/${P}_c5.json)"
    ;;
  flat)
    step 600 gpurun_out/${P}_flat.log python -u bench.py --workload flat
    json gpurun_out/${P}_flat.log
    step 400 gpurun_out/${P}_flat_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_flat -o run \
      --output-format csv -- python -u bench.py --workload flat --no-cpu-baseline
    find gpurun_out/prof_${P}_flat -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${P}_flat_kernel_stats.csv
    rm -rf gpurun_out/prof_${P}_flat
    ;;
  pmc-c4)
    EF=${EF:-373} bash tools/run_pmc.sh gpurun_out/${P}_traffic_c4_10k.json --nq 10000 || exit $?
    ;;
  pmc-c5)
    EF=${EF:-368} bash tools/run_pmc.sh gpurun_out/${P}_traffic_c5_10k.json --workload sq8-ip --nq 10000 || exit $?
    ;;
  pmc-flat)
    bash tools/run_pmc_flat.sh gpurun_out/${P}_traffic_flat.json || exit $?
    ;;
  rehearse8)
    export ALAYA_BENCH_REHEARSE=1
    t0=$(date +%s)
    step 1150 gpurun_out/${P}_rehearse8_c4.log python -u bench.py --gpus 8
    echo "wall_s=$(( $(date +%s) - t0 ))" | tee gpurun_out/${P}_rehearse8_c4.wall
    json gpurun_out/${P}_rehearse8_c4.log
    ;;
  rehearse8-sq8)
    export ALAYA_BENCH_REHEARSE=1
    t0=$(date +%s)
    step 1150 gpurun_out/${P}_rehearse8_c5.log python -u bench.py --gpus 8 --workload sq8-ip --n "${N8_ROWS:-4000000}" --nq "${N8_NQ:-10000}"
    echo "wall_s=$(( $(date +%s) - t0 ))" | tee gpurun_out/${P}_rehearse8_c5.wall
    json gpurun_out/${P}_rehearse8_c5.log
    ;;
  shard-rehearsal)
    wl=${3:-gist}
    step 900 gpurun_out/${P}_shard_rehearsal_$wl.log python -u tools/shard_rehearsal.py --workload "$wl" --nq 10000 \
      --out gpurun_out/${P}_shard_rehearsal_${wl}_10k.json
    ;;
  build-quality)
    step 300 gpurun_out/${P}_gpu_build_tests.log python -u -m pytest tests/test_gpu_build.py -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread
    step 600 gpurun_out/${P}_bq_1m.log python -u tools/build_quality.py --n 1000000 --host
    step 400 gpurun_out/${P}_bq_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${P}_build -o run \
      --output-format csv -- python -u tools/build_quality.py --n 1000000 --efs 400
    find gpurun_out/prof_${P}_build -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${P}_build_kernel_stats.csv
    rm -rf gpurun_out/prof_${P}_build
    ;;
  graph-quality)
    step 600 gpurun_out/${P}_graph_quality_device.log python -u tools/graph_quality.py --graph device \
      --out gpurun_out/${P}_graph_quality_device_gist1m.json
    ;;
  ab-flat)
    for rep in 1 2; do
      for v in $3; do
        if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
        step 200 gpurun_out/${P}_abflat_${v}_$rep.log python -u tools/ab_flat.py --dims ${DIMS:-128}
      done
    done
    ;;
  ab-search)
    wl=$3
    variants=$4
    shift 4
    for rep in 1 2; do
      for v in $variants; do
        if [ "$v" = tree ]; then unset ALAYA_AB_ROOT; else export ALAYA_AB_ROOT=$GRAFT_REPO_ROOT/ab/$v; fi
        step 400 gpurun_out/${P}_ab_${wl}_${v}_$rep.log python -u tools/shape_sweep.py --workload "$wl" "$@"
      done
    done
    ;;
  *)
    echo "unknown recipe: $recipe" >&2
    exit 2
    ;;
esac
