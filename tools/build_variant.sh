#!/bin/bash
# Build a variant of libcnnitmo.so with ONE source recompiled under extra flags
# (for `tools/recipe.sh layers`; CPU side, before a gpurun call):
#   bash tools/build_variant.sh <name> <csrc file.hip | path to another version of it> -DMACRO=value ...
# -> cnn_itmo_amd/lib/variants/lib<name>.so (git-ignored, travels with the tree)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; src=$2; shift 2
O=$R/cnn_itmo_amd/lib/obj
V=$R/cnn_itmo_amd/lib/variants
mkdir -p "$V" /tmp/cnnitmo_var
python -c "import sys; sys.path.insert(0, '$R'); from cnn_itmo_amd import build; build.build(verbose=False)"
base=$(basename "$src" .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I"$R/include" "$@" \
  -I"$R/cnn_itmo_amd/csrc" -c "$( [ -f "$src" ] && echo "$src" || echo "$R/cnn_itmo_amd/csrc/$base.hip" )" \
  -o "/tmp/cnnitmo_var/$name.o"
objs=$(ls $O/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/lib$name.so" $objs "/tmp/cnnitmo_var/$name.o"
echo "$V/lib$name.so"
