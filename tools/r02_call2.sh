source tools/gpu_steps.sh
step 1100 gpurun_out/r02_tests2.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
