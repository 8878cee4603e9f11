#!/bin/bash
# A/B of per-layer timings under an environment switch (GPU box):
#   bash tools/ab_env.sh "<VAR=value>" <layers> <ops>
R=$(cd "$(dirname "$0")/.." && pwd)
for e in "" "$1" "" "$1"; do
  echo "== ${e:-baseline}"
  env $e timeout -k 10 120 python "$R/tools/bench_layers.py" --layers "$2" --ops "$3" --iters 5 | grep -v amdgpu.ids
done
