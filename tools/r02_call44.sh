# last check of the committed build: GPU suite and smoke
source tools/gpu_steps.sh
step 900 gpurun_out/r02_last_gpu_tests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step 300 gpurun_out/r02_last_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
