source tools/gpu_steps.sh
step 600 gpurun_out/r02_time18.log python -u tools/time_fixed.py
