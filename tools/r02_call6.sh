cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/counters_list.txt | sort -u > gpurun_out/sq_counters.txt
wc -l gpurun_out/sq_counters.txt
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex hnsw_search --output-format csv -d gpurun_out/pmc6_$name -o run -- python tools/time_fixed.py --only sift1k,sq8 --reps 3 > gpurun_out/pmc6_$name.log 2>&1 || { echo "pass $name failed"; tail -5 gpurun_out/pmc6_$name.log; }
done
ls -R gpurun_out | head -40
