# flat ring r3: prescan threshold sweep (ALAYA_FLAT_PRESCAN = S samples every S-th row first)
source tools/gpu_steps.sh
for S in 0 16 32 64 128; do
  step 200 gpurun_out/r02_flatpre_$S.log env ALAYA_FLAT_PRESCAN=$S ALAYA_AB_ROOT=$PWD/ab/r3 python -u tools/ab_flat.py --dims 128,64,224
done
grep -H "QPS" gpurun_out/r02_flatpre_*.log
