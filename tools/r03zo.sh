#!/bin/bash
# fp32 transposed-conv forward tiles now that the fp32 3x3 convs run on the halo kernel:
# 128x128 two-per-CU (default) vs 256x128 (CNNITMO_FWD2_BM128=0).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
B="timeout -k 10 300 python3 bench.py --mode infer --dtype float32 --batch 8 --steps 5 --warmup 2 --no-cpu"
for rep in 1 2; do
  $B > gpurun_out/r03zo_base_$rep.json 2> gpurun_out/r03zo_base_$rep.err
  CNNITMO_FWD2_BM128=0 $B > gpurun_out/r03zo_bm256_$rep.json 2> gpurun_out/r03zo_bm256_$rep.err
done
