#!/bin/bash
# wgrad_halo 64x128 block and runtime-occupancy row split: parity, then layer A/Bs.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k conv3x3_fwd_dgrad_wgrad"
$T > gpurun_out/r03v_tests.log 2>&1
CNNITMO_WH_BN128=2 $T >> gpurun_out/r03v_tests.log 2>&1
bash tools/ab_env.sh "CNNITMO_WH_BN128=2" enc3b,enc4a,enc4b,crossa,crossb,dec6,dec7 wgrad > gpurun_out/r03v_ab_bn128.txt 2>&1
bash tools/ab_layers.sh "$R/cnn_itmo_amd/lib/variants/libocc0.so" enc2b,enc3a,enc3b,enc4a,enc4b,crossa,crossb,dec8,dec9b wgrad > gpurun_out/r03v_ab_occ.txt 2>&1
