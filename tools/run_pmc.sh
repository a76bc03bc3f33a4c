#!/bin/bash
# PMC passes for the search kernel at the bench operating point (one counter group per pass,
# kernel-trace only, as MI355X_MICROARCH.md's rocprofv3 section prescribes).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EF=${EF:-400}
ARGS="--ef $EF --steps 5 --warmup 1 --no-cpu-baseline"
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  name=$(echo $grp | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc_$name -o run -- python bench.py $ARGS > gpurun_out/pmc_$name.json 2> gpurun_out/pmc_$name.log || exit $?
done
echo pmc done
