#!/bin/bash
# gpurun with retries ONLY for infrastructure-side transients in which no part of the
# command ran (box prepare failures, busy slots, back-off); any command result ends it.
# usage: tools/gpr.sh <outfile> <timeout> '<command>'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  if grep -q "status=transient\|stopped responding while being prepared\|taken away by the GPU service\|slot(s) on this pod are busy\|backing off" "$out" && ! grep -q "status=ok\|status=fail" "$out"; then
    sleep 45; continue
  fi
  break
done
tail -3 "$out"
