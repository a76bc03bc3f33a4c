source tools/gpu_steps.sh
step 400 gpurun_out/r02_phases_sq8.log python -u tools/profile_phases.py --workload sq8 --n 1000000 --nq 1000 --ef 175
step 400 gpurun_out/r02_phases_sift1k.log python -u tools/profile_phases.py --workload sift --builder gpu --n 1000000 --nq 1000 --ef 85
