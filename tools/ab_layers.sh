#!/bin/bash
# A/B of the per-layer conv timings: the in-tree library vs an experiment build
#   bash tools/ab_layers.sh <exp .so> <layers> <ops>      (GPU box)
R=$(cd "$(dirname "$0")/.." && pwd)
for lib in "$R/cnn_itmo_amd/lib/libcnnitmo.so" "$1" "$R/cnn_itmo_amd/lib/libcnnitmo.so" "$1"; do
  echo "== $(basename $lib)"
  CNNITMO_LIB=$lib timeout -k 10 120 python "$R/tools/bench_layers.py" --layers "$2" --ops "$3" --iters 5 | grep -v amdgpu.ids
done
