#!/bin/bash
# Kernel-trace profile of the default bench (run on the GPU box via gpurun):
#   bash tools/profile_round.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/ (rocprofv3 --kernel-trace --stats) and the bench log.
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$tag" -o run -- \
  python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/prof_${tag}_bench.log" 2>&1
