#!/bin/bash
# Fused dgrad + BN backward: r loaded at the start of the tile's last item (HALO_EARLYR).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CNNITMO_LIB=$V/libearlyr.so $T tests/test_gpu_fold.py tests/test_gpu_ops.py -k "dgrad or fold or bn" > gpurun_out/r03zi_tests.log 2>&1
CNNITMO_LIB=$V/libearlyr.so $T tests/test_gpu_benchshapes.py -k "config2" >> gpurun_out/r03zi_tests.log 2>&1
bash tools/ab_libs.sh enc1b,enc2b,dec6,dec7,dec8,dec9b dgradbn $V/libearlyr.so > gpurun_out/r03zi_ab_earlyr.txt 2>&1
