#!/bin/bash
# Saves a variant build of the package under ab/<name> (git- and gpurun-ignored unless enabled) for
# A/B runs (tools/shape_sweep.py / ab_flat.py / the parity suites with ALAYA_AB_ROOT).  The variant is
# compiled in a copy of the package with extra hipcc flags; the tree's own build is not touched.
# usage: tools/build_ab.sh <name> "<hipcc flags>"
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1
flags=$2
rm -rf "ab/$name" && mkdir -p "ab/$name"
cp -r alayalite_amd "ab/$name/"
rm -rf "ab/$name/alayalite_amd/__pycache__"
# _build.py resolves the sources, the headers (../include) and the outputs from its own location
mkdir -p "ab/$name/include" && cp include/alaya_hip.h "ab/$name/include/"
ALAYA_EXTRA_HIPFLAGS="$flags" python3 -c "
import importlib.util
spec = importlib.util.spec_from_file_location('b', 'ab/$name/alayalite_amd/_build.py')
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b); b.build(force=True)"
rm -rf "ab/$name/alayalite_amd/csrc" "ab/$name/include"
echo "ab/$name: $flags"
