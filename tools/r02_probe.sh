#!/bin/bash
# Round-2 measurement pass (GPU box, via gpurun):
#   per-layer conv table, configs[1] kernel-trace stats, MFMA-busy PMC passes.
#   bash tools/r02_probe.sh <tag>
set -e
tag=$1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
timeout -k 10 240 python3 "$R/tools/bench_layers.py" --ops fwd,dgrad,dgradbn,wgrad --iters 3 > "$O/layers.txt" 2>&1
cd /tmp && export TMPDIR=/tmp
# configs[1]: 1080p b8 fp32 inference, kernel trace
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/infer_trace" -o run -- \
  python3 "$R/bench.py" --mode infer --dtype float32 --batch 8 --infer-batch 0 --no-cpu --steps 5 --warmup 2 \
  > "$O/infer_trace.log" 2>&1
# MFMA busy cycles per kernel (own passes: SQ + GRBM only)
for m in "train --batch 32 --infer-batch 0" "infer --dtype float32 --batch 8 --infer-batch 0"; do
  n=$(echo $m | cut -d' ' -f1)
  timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$O/mfma_$n" -o run -- \
    python3 "$R/bench.py" --mode $m --no-cpu --steps 1 --warmup 1 > "$O/mfma_$n.log" 2>&1
done
