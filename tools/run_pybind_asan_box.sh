#!/bin/bash
# GPU-box script: the pybind module under AddressSanitizer (host code only; the HIP kernels are not
# instrumented), through the public Index API on the GPU.  Build first, in the container:
# tools/build_pybind_asan.sh.  Log: gpurun_out/pybind_asan.log.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/asan_box
ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:abort_on_error=1 timeout -k 10 600 \
  sanitize_build/py_asan tools/sanitize/pybind_driver.py "$GRAFT_REPO_ROOT/sanitize_build/pkg" /tmp/asan_box \
  > gpurun_out/pybind_asan.log 2>&1
rc=$?
tail -20 gpurun_out/pybind_asan.log
exit $rc
