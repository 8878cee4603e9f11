#!/bin/bash
# A/B of the training bench: the in-tree library vs an experiment build (GPU box)
#   bash tools/ab_bench.sh <exp .so> [bench args]
R=$(cd "$(dirname "$0")/.." && pwd)
exp=$1; shift
for lib in "$R/cnn_itmo_amd/lib/libcnnitmo.so" "$exp" "$R/cnn_itmo_amd/lib/libcnnitmo.so" "$exp"; do
  echo "== $(basename $lib)"
  CNNITMO_LIB=$lib timeout -k 10 300 python "$R/bench.py" --no-cpu "$@" 2>&1 | grep -E '^\{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['achieved'])"
done
