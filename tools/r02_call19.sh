source tools/gpu_steps.sh
step 1000 gpurun_out/r02_tests19.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf
step 120 gpurun_out/r02_smoke19.log python -c "import __graft_entry__ as g; g.smoke()"
