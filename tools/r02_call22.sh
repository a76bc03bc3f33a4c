# fine-grained phase stamps (diagnostic build ab/fine) + per-query tail statistics, then the same
# tail statistics from the production build's coarse stamps
source tools/gpu_steps.sh
export ALAYA_AB_ROOT=$PWD/ab/fine
step 400 gpurun_out/r02_fine_sift.log python -u tools/profile_phases.py --workload sift --builder gpu --ef 85 --nq 1000 --fine
step 400 gpurun_out/r02_fine_sq8.log python -u tools/profile_phases.py --workload sq8 --ef 175 --nq 1000 --fine
step 500 gpurun_out/r02_fine_gist.log python -u tools/profile_phases.py --workload gist --builder gpu --ef 387 --nq 1000 --fine


