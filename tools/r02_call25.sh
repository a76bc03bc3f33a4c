# SQ8 occupancy A/B: base (row-major, 426 VGPRs) vs chunk-major (ab/cm) vs chunk-major + 2 waves/EU
source tools/gpu_steps.sh
step 400 gpurun_out/r02_sq8ab_new.log python -u tools/ab_sq8.py --hash 0,14,13,12,11
ALAYA_AB_ROOT=$PWD/ab/cm step 400 gpurun_out/r02_sq8ab_cm.log python -u tools/ab_sq8.py --hash 0,14,13,12,11
ALAYA_AB_ROOT=$PWD/ab/base step 400 gpurun_out/r02_sq8ab_base.log python -u tools/ab_sq8.py --hash 0,14,13,12,11
grep -h "engine\|QPS" gpurun_out/r02_sq8ab_*.log
