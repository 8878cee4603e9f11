#!/bin/bash
# tconv_ws probes (old kernel: no stores / L2-resident A) and the 256-column up8 forward.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CNNITMO_TWS_BN256=1 $T tests/test_gpu_ops.py -k "tconv" > gpurun_out/r03y_tests.log 2>&1
CNNITMO_TWS_BN256=1 $T tests/test_gpu_benchshapes.py >> gpurun_out/r03y_tests.log 2>&1
bash tools/ab_env.sh "CNNITMO_TWS_BN256=1" up8 fwd > gpurun_out/r03y_ab_bn256.txt 2>&1
bash tools/ab_libs.sh up6,up7,up8 fwd $V/libtws_nostore.so $V/libtws_fixeda.so $V/libtws_both.so > gpurun_out/r03y_ab_tws_probe.txt 2>&1
