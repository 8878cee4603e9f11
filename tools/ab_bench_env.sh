#!/bin/bash
# A/B of the training bench under an environment switch (GPU box):
#   bash tools/ab_bench_env.sh "<VAR=value>" [bench args]
R=$(cd "$(dirname "$0")/.." && pwd)
sw=$1; shift
for e in "" "$sw" "" "$sw"; do
  echo "== ${e:-baseline}"
  env $e timeout -k 10 300 python "$R/bench.py" --no-cpu "$@" 2>&1 | grep -E '^\{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
