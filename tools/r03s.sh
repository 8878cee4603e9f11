set -e
R=$GRAFT_REPO_ROOT

for i in 1 2; do
for v in base wsold; do
  lib=$R/cnn_itmo_amd/lib/variants/lib$v.so; [ $v = base ] && lib=$R/cnn_itmo_amd/lib/libcnnitmo.so
  echo "== $v"; CNNITMO_LIB=$lib timeout -k 10 120 python tools/bench_layers.py --layers up6,up7,up8 --ops fwd --iters 5 2>&1 | grep -v amdgpu.ids
done
done
