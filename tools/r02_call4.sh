source tools/gpu_steps.sh
step 300 gpurun_out/r02_pipe_tests.log python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step 900 gpurun_out/r02_tests4.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step 600 gpurun_out/r02_time4.log python -u tools/time_fixed.py
