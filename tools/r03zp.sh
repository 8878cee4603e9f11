#!/bin/bash
# fp32 weight-stationary Conv2DTranspose forward for inference (CNNITMO_TCONV_WS_F32=1).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export CNNITMO_TCONV_WS_F32=1
$T tests/test_golden.py -k "gpu" > gpurun_out/r03zp_tests.log 2>&1
$T tests/test_gpu_benchshapes.py -k "config1 or northstar or small_frame" >> gpurun_out/r03zp_tests.log 2>&1
$T tests/test_gpu_tiled.py tests/test_gpu_model.py tests/test_gpu_ops.py >> gpurun_out/r03zp_tests.log 2>&1
B="timeout -k 10 300 python3 bench.py --mode infer --dtype float32 --batch 8 --steps 5 --warmup 2 --no-cpu"
for rep in 1 2; do
  CNNITMO_TCONV_WS_F32=0 $B > gpurun_out/r03zp_base_$rep.json 2> gpurun_out/r03zp_base_$rep.err
  CNNITMO_TCONV_WS_F32=1 $B > gpurun_out/r03zp_ws_$rep.json 2> gpurun_out/r03zp_ws_$rep.err
done
