# config 5 at 10k queries: visited-table size vs residency.  base: 32 ef-slot tables (3 waves/CU at ef 340),
# tree: tables halved until one wave per SIMD fits (4 waves/CU); base with a forced 2^13 table for reference
source tools/gpu_steps.sh
step 1000 gpurun_out/r02_c5_hash_new.log python -u tools/ab_sq8.py --n 10000000 --ef 340 --nq 1000,10000 --hash 0 --reps 5
ALAYA_AB_ROOT=$PWD/ab/base step 1000 gpurun_out/r02_c5_hash_base.log python -u tools/ab_sq8.py --n 10000000 --ef 340 --nq 1000,10000 --hash 0,13 --reps 5
grep -H QPS gpurun_out/r02_c5_hash_*.log
