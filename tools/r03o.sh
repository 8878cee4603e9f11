#!/bin/bash
# Full GPU suite, then the default bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > gpurun_out/r03o_pytest.log 2>&1
tail -3 gpurun_out/r03o_pytest.log
timeout -k 10 600 python3 bench.py > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err
