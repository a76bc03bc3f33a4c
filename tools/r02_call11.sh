source tools/gpu_steps.sh
step 900 gpurun_out/r02_tests11.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
step 600 gpurun_out/r02_time11.log python -u tools/time_fixed.py --visited 0
