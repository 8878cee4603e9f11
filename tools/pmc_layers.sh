#!/bin/bash
# Per-layer PMC passes of the conv kernels (GPU box, via gpurun), one pass per
# counter group (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE never share a pass):
#   bash tools/pmc_layers.sh <tag> <layers> <ops>
# Post-process with tools/pmc_summary.py gpurun_out/<tag>.
set -e
tag=$1; layers=$2; ops=$3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/p$i" -o run -- \
    python3 "$R/tools/bench_layers.py" --layers "$layers" --ops "$ops" --iters 1 > "$O/p$i.log" 2>&1
  i=$((i+1))
done
