#!/bin/bash
# round-3: tconv_stream launch-level BN sums (parity + bench), wgrad rows-per-step A/B
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_benchshapes.py tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 500 --timeout-method thread > $O/r03g_tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --infer-batch 0 --k4-batch 0 --ns-batch 0 > $O/r03g_bench.json 2> $O/r03g_bench.err
timeout -k 10 400 bash tools/ab_libs.sh dec6,dec7,dec8,dec9 wgrad cnn_itmo_amd/lib/variants/libwhr3d2.so cnn_itmo_amd/lib/variants/libwhr4d1.so > $O/r03g_ab_whrows.txt 2>&1
