source tools/gpu_steps.sh
ALAYA_FLAT_WS0=1 step 300 gpurun_out/r02_order_old.log python -u -m pytest tests/test_flat.py::test_flat_exact tests/test_contracts_gpu.py::test_two_streams_one_index -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step 300 gpurun_out/r02_order_ws.log python -u -m pytest tests/test_flat.py::test_flat_exact tests/test_contracts_gpu.py::test_two_streams_one_index -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step 300 gpurun_out/r02_order_torchfirst.log python -u -m pytest tests/test_contracts_gpu.py::test_two_streams_one_index tests/test_flat.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
