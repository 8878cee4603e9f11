#!/bin/bash
# Current build: full GPU suite (incl. the one-rank RCCL path), default bench.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA -k "rccl" > gpurun_out/r03x_rccl.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x_gpu_tests.log 2>&1
timeout -k 10 600 python3 bench.py > gpurun_out/r03x_bench.json 2> gpurun_out/r03x_bench.err
