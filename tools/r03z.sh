#!/bin/bash
# tconv_ws whole-line stores (line_pair) vs 64-B segments; 256-column up8 forward.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T tests/test_gpu_ops.py -k "tconv" > gpurun_out/r03z_tests.log 2>&1
CNNITMO_TWS_BN256=1 $T tests/test_gpu_ops.py -k "tconv" >> gpurun_out/r03z_tests.log 2>&1
CNNITMO_TWS_BN256=1 $T tests/test_gpu_benchshapes.py -k "config2" >> gpurun_out/r03z_tests.log 2>&1
bash tools/ab_libs.sh up6,up7,up8 fwd,dgrad $V/libtws_nolines.so > gpurun_out/r03z_ab_lines.txt 2>&1
CNNITMO_TWS_BN256=1 bash tools/ab_libs.sh up8 fwd $V/libtws_nolines.so > gpurun_out/r03z_ab_lines_bn256.txt 2>&1
CNNITMO_LIB=$V/libhalo_lines.so $T tests/test_gpu_ops.py -k "conv3x3" >> gpurun_out/r03z_tests.log 2>&1
bash tools/ab_libs.sh enc2b,dec6,dec8,dec9 fwd,dgrad $V/libhalo_lines.so > gpurun_out/r03z_ab_halo_lines.txt 2>&1
CNNITMO_FWD2_256=1 $T tests/test_gpu_ops.py -k "tconv" >> gpurun_out/r03z_tests.log 2>&1
bash tools/ab_env.sh "CNNITMO_FWD2_256=1" up6,up7 dgrad > gpurun_out/r03z_ab_fwd2_256.txt 2>&1
