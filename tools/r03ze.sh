#!/bin/bash
# enc1b weight gradient (32x32 block, HBM-bound): 64-pixel strips with 2/4/6 row groups in flight.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
V=$R/cnn_itmo_amd/lib/variants
T="timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for lib in $V/libahead4.so $V/libahead6.so; do
  CNNITMO_WH_TW128=0 CNNITMO_LIB=$lib $T tests/test_gpu_ops.py -k "conv3x3_fwd_dgrad_wgrad" >> gpurun_out/r03ze_tests.log 2>&1
done
for rep in 1 2; do
  echo "== base (TW 128)"; timeout -k 10 120 python tools/bench_layers.py --layers enc1b --ops wgrad --iters 5 | grep -v amdgpu
  echo "== base TW 64"; CNNITMO_WH_TW128=0 timeout -k 10 120 python tools/bench_layers.py --layers enc1b --ops wgrad --iters 5 | grep -v amdgpu
  for d in 4 6; do
    echo "== TW 64 ahead $d"; CNNITMO_WH_TW128=0 CNNITMO_LIB=$V/libahead$d.so timeout -k 10 120 python tools/bench_layers.py --layers enc1b --ops wgrad --iters 5 | grep -v amdgpu
  done
done > gpurun_out/r03ze_ab_enc1b_wgrad.txt 2>&1
