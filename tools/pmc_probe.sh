#!/bin/bash
# PMC probe of one conv op (GPU box):  bash tools/pmc_probe.sh <tag> <layer> <op> "<counters>"
set -e
tag=$1; layer=$2; op=$3; ctr=$4
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_$tag" -o run -- \
  python3 "$R/tools/bench_layers.py" --layers "$layer" --ops "$op" --iters 1 > "$R/gpurun_out/pmc_${tag}.log" 2>&1
