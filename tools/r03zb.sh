#!/bin/bash
# tconv_stream (up9 forward) whole-line stores: parity, A/B against 64-B segments.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T tests/test_gpu_ops.py -k "tconv" > gpurun_out/r03zb_tests.log 2>&1
$T tests/test_gpu_benchshapes.py -k "config2" >> gpurun_out/r03zb_tests.log 2>&1
bash tools/ab_libs.sh up9 fwd $V/libts_nolines.so > gpurun_out/r03zb_ab_ts_lines.txt 2>&1
