#!/bin/bash
# Per-layer timings of several library builds, interleaved twice (GPU box):
#   bash tools/ab_libs.sh <layers> <ops> <lib.so>...
R=$(cd "$(dirname "$0")/.." && pwd)
L=$1; O=$2; shift 2
for rep in 1 2; do
  for lib in "$R/cnn_itmo_amd/lib/libcnnitmo.so" "$@"; do
    echo "== $(basename $lib)"
    CNNITMO_LIB=$lib timeout -k 10 120 python "$R/tools/bench_layers.py" --layers "$L" --ops "$O" --iters 5 | grep -v amdgpu.ids
  done
done
