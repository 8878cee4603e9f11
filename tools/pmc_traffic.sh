#!/bin/bash
# HBM traffic per kernel from PMC counters (GPU box, via gpurun), one counter per
# pass as MI355X_MICROARCH.md prescribes (FETCH_SIZE and WRITE_SIZE cannot share
# a pass); a 1-step bench run.  Post-process locally with tools/pmc_traffic.py.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_$c" -o run -- \
    python3 "$R/bench.py" --no-cpu --steps 1 --warmup 0 --k4-batch 0 > "$R/gpurun_out/pmc_$c.log" 2>&1
done
