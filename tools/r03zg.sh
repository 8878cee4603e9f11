#!/bin/bash
# 32x32 wgrad at one wave per kernel row by default: full GPU suite; 64x32 (enc2a) layout A/B; bench.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CNNITMO_LIB=$V/libwm1.so $T tests/test_gpu_ops.py -k "conv3x3_fwd_dgrad_wgrad" > gpurun_out/r03zg_tests.log 2>&1
bash tools/ab_libs.sh enc2a wgrad $V/libwm1.so > gpurun_out/r03zg_ab_enc2a_wm1.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03zg_gpu_tests.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/r03zg_bench.json 2> gpurun_out/r03zg_bench.err
