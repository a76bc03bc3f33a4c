#!/bin/bash
# ASAN and TSAN runs of the engine's host C++: the host translation units (capi.cpp,
# hnsw_build.cpp, graph_update.cpp + the driver tools/sanitize/host_checks.cpp) are compiled with
# -fsanitize=address / -fsanitize=thread; the HIP kernel objects are linked uninstrumented.  Then the
# pybind module (pybind_module.cpp) under ASan: tools/build_pybind_asan.sh builds an instrumented copy
# of the package and an ASan-linked embedded python, and tools/sanitize/pybind_driver.py runs its
# host-only surface here (the Index API half runs on the GPU box: tools/run_pybind_asan_box.sh).
# Logs go to profiles/r03/sanitizers/.  CPU only.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=profiles/r03/sanitizers
B=$(mktemp -d)
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CS=alayalite_amd/csrc
HOST_SRC="$CS/capi.cpp $CS/hnsw_build.cpp $CS/graph_update.cpp tools/sanitize/host_checks.cpp"
# device objects (no sanitizer)
for f in search_kernels build_kernels flat_kernels; do
  "$HIPCC" -O2 -std=c++17 -fPIC -ffp-contract=off -x hip --offload-arch=gfx950 -Iinclude -c "$CS/$f.hip" -o "$B/$f.o"
done
DEV_OBJS="$B/search_kernels.o $B/build_kernels.o $B/flat_kernels.o"
HOSTFLAGS="-std=c++17 -g -O1 -fno-omit-frame-pointer -ffp-contract=off -pthread -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
for san in address thread; do
  objs=""
  for s in $HOST_SRC; do
    o="$B/$(basename "$s" .cpp)_$san.o"
    g++ $HOSTFLAGS -fsanitize=$san -c "$s" -o "$o"
    objs="$objs $o"
  done
  g++ -fsanitize=$san -pthread -o "$B/host_checks_$san" $objs $DEV_OBJS -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
  if [ "$san" = address ]; then
    ASAN_OPTIONS=detect_leaks=1:abort_on_error=1:verify_asan_link_order=0 "$B/host_checks_$san" --hip "$B" \
      > "$OUT/asan.log" 2>&1 && echo "asan: clean" || { echo "asan: FAILED"; tail -30 "$OUT/asan.log"; exit 1; }
  else
    TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$B/host_checks_$san" --no-hip "$B" \
      > "$OUT/tsan.log" 2>&1 && echo "tsan: clean" || { echo "tsan: FAILED"; tail -40 "$OUT/tsan.log"; exit 1; }
  fi
done
rm -rf "$B"
bash tools/build_pybind_asan.sh > "$OUT/pybind_asan_build.log" 2>&1
mkdir -p /tmp/pybind_asan_cpu
ASAN_OPTIONS=detect_leaks=0:alloc_dealloc_mismatch=0:abort_on_error=1 sanitize_build/py_asan \
  tools/sanitize/pybind_driver.py "$PWD/sanitize_build/pkg" /tmp/pybind_asan_cpu > "$OUT/pybind_asan_cpu.log" 2>&1 \
  && echo "pybind asan (host surface): clean" || { echo "pybind asan: FAILED"; tail -30 "$OUT/pybind_asan_cpu.log"; exit 1; }
