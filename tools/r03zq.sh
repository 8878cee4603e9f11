#!/bin/bash
# fp32 halo forward by default: full GPU suite, then the final evidence pass
# (PMC traffic per shape, kernel-trace profile, default bench) of this build.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03zq_gpu_tests.log 2>&1
bash "$R/tools/pmc_traffic.sh"
bash "$R/tools/profile_round.sh" r03zq --steps 5 --warmup 2 --infer-batch 0 --ns-batch 0 --k4-batch 0
cd "$R"
timeout -k 10 600 python3 bench.py > gpurun_out/r03zq_bench.json 2> gpurun_out/r03zq_bench.err
