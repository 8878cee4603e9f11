#!/bin/bash
# round-3: split level-0 concat -- parity (full-size checker + model tests), then bench A/B
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_benchshapes.py tests/test_gpu_model.py tests/test_gpu_fold.py tests/test_gpu_tiled.py -x -v -s --timeout 500 --timeout-method thread > $O/r03d_tests.log 2>&1
timeout -k 10 600 bash tools/ab_bench_env.sh "CNNITMO_SPLIT_CAT=0" --infer-batch 0 --k4-batch 0 --ns-batch 0 --steps 10 > $O/r03d_ab_splitcat.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --infer-batch 0 --k4-batch 0 --ns-batch 0 > $O/r03d_bench.json 2> $O/r03d_bench.err
