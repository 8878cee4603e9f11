set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "first_layer" 2>&1 | tail -3
for i in 1 2; do
for v in base c3old; do
  lib=$R/cnn_itmo_amd/lib/variants/lib$v.so; [ $v = base ] && lib=$R/cnn_itmo_amd/lib/libcnnitmo.so
  echo "== $v"; CNNITMO_LIB=$lib timeout -k 10 120 python tools/probe_c3.py 2>&1 | grep -v amdgpu.ids
done
done
