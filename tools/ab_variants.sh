#!/bin/bash
# Per-layer timings of the in-tree library and of experiment builds (GPU box):
#   bash tools/ab_variants.sh <layers> <ops> <lib.so>...
R=$(cd "$(dirname "$0")/.." && pwd)
layers=$1; ops=$2; shift 2
for lib in "$R/cnn_itmo_amd/lib/libcnnitmo.so" "$@"; do
  echo "== $(basename $lib)"
  CNNITMO_LIB=$lib timeout -k 10 120 python "$R/tools/bench_layers.py" --layers "$layers" --ops "$ops" --iters 5 | grep -v amdgpu.ids
done
