#!/bin/bash
# Issue/wait attribution of a conv kernel's wave cycles (GPU box, via gpurun): four
# rocprofv3 --pmc passes (<= 8 SQ counters + GRBM_GUI_ACTIVE each) over tools/bench_layers.py
#   bash tools/pmc_attrib.sh <tag> <layers> <ops> [bench_layers args...]
# Post-process: python tools/pmc_attrib.py gpurun_out/attrib_<tag> [kernel-name filter]
set -e -o pipefail
tag=$1; layers=$2; ops=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/attrib_$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/p$i" -o run -- \
    python3 "$R/tools/bench_layers.py" --layers "$layers" --ops "$ops" --iters 2 "$@" > "$O/p$i.log" 2>&1
  i=$((i+1))
done
echo "attrib $tag: $i passes"
