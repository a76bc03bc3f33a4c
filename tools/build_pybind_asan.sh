#!/bin/bash
# Builds the AddressSanitizer copy of the package for the pybind-module runs (CPU only, no GPU):
#   sanitize_build/pkg/alayalite_amd/  -- the Python sources, libalaya_hip.so with its host
#       translation units (capi, hnsw_build, graph_update) instrumented and the HIP kernel objects
#       not, and _alayalitepy*.so (pybind_module.cpp) instrumented;
#   sanitize_build/py_asan  -- python3 embedded in an ASan-linked main (tools/sanitize/py_asan_main.cpp),
#       so the runtime comes first without LD_PRELOAD.
# The directory is git-ignored; it travels to the GPU box with the tree (tools/run_pybind_asan_box.sh).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=sanitize_build
PKG=$OUT/pkg/alayalite_amd
rm -rf "$OUT"
mkdir -p "$PKG" "$OUT/obj"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CS=alayalite_amd/csrc
SAN="-fsanitize=address -fno-omit-frame-pointer"
for f in search_kernels build_kernels flat_kernels; do
  "$HIPCC" -O2 -std=c++17 -fPIC -ffp-contract=off -x hip --offload-arch=gfx950 -Iinclude -c "$CS/$f.hip" -o "$OUT/obj/$f.o" &
done
wait
HOSTFLAGS="-std=c++17 -g -O1 -fPIC -ffp-contract=off -pthread -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__"
for f in capi hnsw_build graph_update; do
  g++ $HOSTFLAGS $SAN -c "$CS/$f.cpp" -o "$OUT/obj/$f.o"
done
g++ -shared $SAN -pthread -o "$PKG/libalaya_hip.so" "$OUT"/obj/*.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYBIND=$(python3 -c "import pybind11;print(pybind11.get_include())")
PYINC=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
g++ -std=c++17 -g -O1 -shared -fPIC $SAN -ffp-contract=off -fvisibility=hidden -I"$PYBIND" -I"$PYINC" -Iinclude \
  "$CS/pybind_module.cpp" -o "$PKG/_alayalitepy$EXT" -L"$PKG" -lalaya_hip -Wl,-rpath,'$ORIGIN'
cp alayalite_amd/*.py "$PKG/"
g++ $SAN -g -O1 $(python3-config --includes) tools/sanitize/py_asan_main.cpp -o "$OUT/py_asan" \
  $(python3-config --ldflags --embed)
rm -rf "$OUT/obj"
echo "built $OUT"
