#!/bin/bash
# 64x128 wgrad blocks by default: full GPU suite, 64x64 two-rows A/B, default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w_gpu_tests.log 2>&1
bash tools/ab_layers.sh "$R/cnn_itmo_amd/lib/variants/librows64.so" enc2b,enc3a,dec9b wgrad > gpurun_out/r03w_ab_rows64.txt 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err
