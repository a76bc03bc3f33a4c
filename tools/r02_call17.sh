source tools/gpu_steps.sh
step 900 gpurun_out/r02_tests17.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
step 600 gpurun_out/r02_time17.log python -u tools/time_fixed.py
