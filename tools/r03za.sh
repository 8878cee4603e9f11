#!/bin/bash
# Whole-line tconv_ws stores + 256x256 tconv dgrad tiles by default: full GPU suite, bench.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03za_gpu_tests.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/r03za_bench.json 2> gpurun_out/r03za_bench.err
