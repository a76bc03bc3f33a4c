#!/bin/bash
# GPU-box script: SQ instruction / cycle counters of the search kernel at a batch shape (issue
# budget per expansion), one counter group per pass, kernel-trace only (MI355X_MICROARCH.md's
# rocprofv3 rules: <= 8 SQ and <= 2 GRBM counters a pass, no --pmc with other trace domains).
# usage: WORKLOAD=sift NQ=10000 [EF=70] bash tools/run_pmc_sq.sh    -> gpurun_out/pmc_sq_<workload>_<nq>_*/
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
W=${WORKLOAD:-sift}
NQ=${NQ:-10000}
EFARG=""
if [ -n "$EF" ]; then EFARG="--ef $EF"; fi
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"
i=0
for grp in "$P1" "$P2"; do
  i=$((i + 1))
  out=gpurun_out/pmc_sq_${W}_${NQ}_p$i
  rm -rf $out
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex hnsw_search_kernel --output-format csv -d $out -o run -- python -u tools/shape_sweep.py --workload $W --nq $NQ --reps 5 $EFARG > $out.txt 2>&1 || { tail -5 $out.txt; exit 1; }
  tail -1 $out.txt
  find $out -name "*kernel_trace.csv" -delete
done
echo pmc sq done
