"""Data-parallel path on the GPU: two ranks share the box's one GPU
over gloo (tools/dp_rehearsal.py) and run the real engine with the bucketed
gradient all-reduce launched during backward.  Every rank must end with
bit-identical parameters equal to a single-process replay that averages the
ranks' gradients itself.  (RCCL itself needs one GPU per rank: the driver's
8-GPU bench exercises it; this checks the bucketing, stream ordering and
averaging.)"""
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_dp_two_ranks_one_gpu(dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, CNNITMO_DEVICE="0", CNNITMO_DIST_BACKEND="gloo", DTYPE=dtype,
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    port = str(29600 + (os.getpid() % 200) + (1 if dtype == "bfloat16" else 0) * 300)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.join(ROOT, "tools", "dp_rehearsal.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ranks identical" in r.stdout
