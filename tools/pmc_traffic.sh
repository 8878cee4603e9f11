#!/bin/bash
# HBM traffic per kernel from PMC counters (GPU box, via gpurun), one counter per
# pass as MI355X_MICROARCH.md prescribes (FETCH_SIZE and WRITE_SIZE cannot share
# a pass); one bench step per workload shape.  Post-process locally with
#   python tools/pmc_traffic.py gpurun_out profiles/pmc_traffic.json
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
sha256sum "$R/cnn_itmo_amd/lib/libcnnitmo.so" | cut -c1-16 > "$R/gpurun_out/pmc_lib_sha.txt"
run() {  # tag shape-key bench-args...
  local tag=$1 shape=$2
  shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "$shape" > "$R/gpurun_out/pmc_${tag}_$c.shape"
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_${tag}_$c" -o run -- \
      python3 "$R/bench.py" --no-cpu --steps 1 --warmup 0 --k4-batch 0 --infer-batch 0 --ns-batch 0 --f32-train-batch 0 "$@" \
      > "$R/gpurun_out/pmc_${tag}_$c.log" 2>&1
  done
}
run train "train 1080x1920 b32 bfloat16"
run infer8 "infer 1080x1920 b8 float32" --mode infer --dtype float32 --batch 8
run infer32 "infer 1080x1920 b32 float32" --mode infer --dtype float32 --batch 32
run train4k "train 2160x3840 b8 bfloat16" --height 2160 --width 3840 --batch 8
run train32 "train 1080x1920 b8 float32" --dtype float32 --batch 8
