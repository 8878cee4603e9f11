set -e
R=$GRAFT_REPO_ROOT
for i in 1 2; do
for v in base c3nostore c3noload c3rpb8 c3rpb2; do
  lib=$R/cnn_itmo_amd/lib/variants/lib$v.so; [ $v = base ] && lib=$R/cnn_itmo_amd/lib/libcnnitmo.so
  echo "== $v"; CNNITMO_LIB=$lib timeout -k 10 120 python tools/probe_c3.py 2>&1 | grep -v amdgpu.ids
done
done
