set -e
R=$GRAFT_REPO_ROOT
for v in whr2 c3old; do
  echo "== $v"
  CNNITMO_LIB=$R/cnn_itmo_amd/lib/variants/lib$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_benchshapes.py -k config2 > gpurun_out/r03p_$v.log 2>&1 || true
  tail -2 gpurun_out/r03p_$v.log
done
