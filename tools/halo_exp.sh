#!/bin/bash
# Timing-only experiment libraries of the halo kernel (HALO_EXP in conv_halo.hip):
#   bash tools/halo_exp.sh build        (here: compiles exp/libcnnitmo_expN.so, N = 1..4)
#   bash tools/halo_exp.sh run <layers> (GPU box: bench_layers fwd with each library)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = build ]; then
  python -c "import sys; sys.path.insert(0, '$R'); from cnn_itmo_amd import build as B; B.build(jobs=8)"
  mkdir -p "$R/exp"
  objs=$(ls "$R"/cnn_itmo_amd/lib/obj/*.o | grep -v conv_halo.o)
  for n in 1 2 3 4 5 6 7; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DHALO_EXP=$n -I"$R/include" \
      -c "$R/cnn_itmo_amd/csrc/conv_halo.hip" -o "$R/exp/conv_halo_$n.o" &
  done
  wait
  for n in 1 2 3 4 5 6 7; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/exp/libcnnitmo_exp$n.so" $objs "$R/exp/conv_halo_$n.o"
  done
else
  L=${2:-dec9}
  for n in 0 1 2 3 4 5 6 7 7; do
    lib="$R/cnn_itmo_amd/lib/libcnnitmo.so"; [ $n -gt 0 ] && lib="$R/exp/libcnnitmo_exp$n.so"
    echo "== HALO_EXP=$n"
    CNNITMO_LIB=$lib timeout -k 10 120 python "$R/tools/bench_layers.py" --layers "$L" --ops ${OPS:-fwd,dgrad} --iters 5 | grep -E "fwd|dgrad"
  done
fi
