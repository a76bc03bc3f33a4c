#!/bin/bash
# Saves a variant build of the package under ab/<name> (git- and gpurun-ignored unless enabled) for
# A/B runs (tools/shape_sweep.py / time_fixed.py with ALAYA_AB_ROOT): usage tools/build_ab.sh <name> "<hipcc flags>"
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1
flags=$2
ALAYA_EXTRA_HIPFLAGS="$flags" python3 -c "
import importlib.util
spec = importlib.util.spec_from_file_location('b', 'alayalite_amd/_build.py')
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b); b.build(force=True)"
rm -rf "ab/$name" && mkdir -p "ab/$name"
cp -r alayalite_amd "ab/$name/"
rm -rf "ab/$name/alayalite_amd/csrc" "ab/$name/alayalite_amd/__pycache__"
# restore the tree's default build
python3 -c "
import importlib.util
spec = importlib.util.spec_from_file_location('b', 'alayalite_amd/_build.py')
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b); b.build(force=True)"
echo "ab/$name: $flags"
