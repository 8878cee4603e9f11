#!/bin/bash
# enc1b weight gradient: one wave per kernel row across the 32x32 block (WH_WN32=1).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
CNNITMO_LIB=$V/libwn1.so $T tests/test_gpu_ops.py -k "conv3x3_fwd_dgrad_wgrad" > gpurun_out/r03zf_tests.log 2>&1
CNNITMO_WH_TW128=0 CNNITMO_LIB=$V/libwn1a4.so $T tests/test_gpu_ops.py -k "conv3x3_fwd_dgrad_wgrad" >> gpurun_out/r03zf_tests.log 2>&1
B="timeout -k 10 120 python tools/bench_layers.py --layers enc1b --ops wgrad --iters 5"
for rep in 1 2; do
  echo "== base (TW 128, 6 waves)"; $B | grep -v amdgpu
  echo "== wn1 TW 128"; CNNITMO_LIB=$V/libwn1.so $B | grep -v amdgpu
  echo "== wn1 TW 64"; CNNITMO_WH_TW128=0 CNNITMO_LIB=$V/libwn1.so $B | grep -v amdgpu
  echo "== wn1 TW 64 ahead 4"; CNNITMO_WH_TW128=0 CNNITMO_LIB=$V/libwn1a4.so $B | grep -v amdgpu
done > gpurun_out/r03zf_ab_enc1b_wn1.txt 2>&1
