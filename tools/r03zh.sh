#!/bin/bash
# Round-3 final evidence pass: PMC traffic per shape, kernel-trace profile of the
# default bench, then the default bench line itself (same library build throughout).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/tools/pmc_traffic.sh"
bash "$R/tools/profile_round.sh" r03zh --steps 5 --warmup 2 --infer-batch 0 --ns-batch 0 --k4-batch 0
cd "$R"
timeout -k 10 600 python3 bench.py > gpurun_out/r03zh_bench.json 2> gpurun_out/r03zh_bench.err
