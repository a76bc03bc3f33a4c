source tools/gpu_steps.sh
step 300 gpurun_out/r02_ws_tests.log python -u -m pytest tests/test_two_wave_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step 600 gpurun_out/r02_time16.log python -u tools/time_fixed.py --ws 0,1 --only sift1k,sq8,sift
