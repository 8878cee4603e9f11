#!/bin/bash
# Fused dgrad + BN backward: r lines touched into L2 one item before the epilogue (HALO_RPF).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CNNITMO_LIB=$V/librpf.so $T tests/test_gpu_fold.py tests/test_gpu_ops.py -k "dgrad or fold or bn" > gpurun_out/r03zd_tests.log 2>&1
CNNITMO_LIB=$V/librpf.so $T tests/test_gpu_benchshapes.py -k "config2" >> gpurun_out/r03zd_tests.log 2>&1
bash tools/ab_libs.sh enc1b,enc2b,dec6,dec7,dec8,dec9b dgradbn $V/librpf.so > gpurun_out/r03zd_ab_rpf.txt 2>&1
