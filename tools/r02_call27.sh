# flat scan A/B: base (HEAD) vs B (branch-free tile loads + row norms a step ahead) vs C (B + two tiles in flight)
source tools/gpu_steps.sh
step 300 gpurun_out/r02_flatab_base.log env ALAYA_AB_ROOT=$PWD/ab/base python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatab_b.log env ALAYA_AB_ROOT=$PWD/ab/b python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatab_c.log env ALAYA_AB_ROOT=$PWD/ab/c python -u tools/ab_flat.py --dims 128,64,224
step 300 gpurun_out/r02_flatab_base2.log env ALAYA_AB_ROOT=$PWD/ab/base python -u tools/ab_flat.py --dims 128
grep -h "engine\|QPS" gpurun_out/r02_flatab_*.log
