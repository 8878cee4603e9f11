"""Data-parallel path on the GPU: two ranks share the box's one GPU
over gloo and run the real engine with the bucketed gradient all-reduce launched
during backward.

* ``tools/dp_rehearsal.py`` trains through the public path
  (``Model.fit_generator(..., distributed=True)`` over rank-sharded, zip-paired
  ImageDataGenerator streams): every rank must end with bit-identical parameters
  and moving statistics equal to a single-process replay at the global batch.
* ``bench.py --gpus 2`` must start its two ranks by itself (no torchrun
  environment), report ``n_gpus == 2`` / ``dp2`` and identical replicas.

RCCL refuses two ranks on one GPU, so on this box the RCCL path runs as a one-rank
``nccl`` group with CNNITMO_DIST_FORCE=1 (``tools/rccl_world1.py``): the broadcast,
the bucketed all-reduces launched during backward and the moving-statistics
all-reduce execute in RCCL, and the result must be bit-identical to training without
collectives.  The driver's multi-GPU bench runs it across GPUs."""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    return dict(os.environ, CNNITMO_DEVICE="0", CNNITMO_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", **kw)


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_dp_two_ranks_one_gpu(dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = str(29600 + (os.getpid() % 200) + (1 if dtype == "bfloat16" else 0) * 300)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.join(ROOT, "tools", "dp_rehearsal.py")]
    r = subprocess.run(cmd, env=_env(DTYPE=dtype), capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ranks identical" in r.stdout
    assert r.stdout.count("Model.fit") == 2, r.stdout  # 11 frames (ragged tail) and 9 (tail dropped)
    print("\n".join(r.stdout.strip().splitlines()[-3:]))


def test_bench_spawns_ranks():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--height", "64", "--width", "96",
           "--batch", "2", "--steps", "2", "--warmup", "1", "--no-cpu", "--infer-batch", "1", "--bucket-mb", "0.5", "--k4-batch", "1", "--k4-steps", "1",
           "--f32-train-batch", "1", "--f32-train-steps", "1",
           "--ns-batch", "2"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 4
    assert res["replicas"]["identical"], res["replicas"]
    assert res["allreduce_exposed"]["world_size"] == 2
    assert res["allreduce_exposed"]["buckets"] >= 2
    assert res["fp32_infer"]["config"]["global_batch"] == 2
    assert res["fp32_infer_b32"]["config"]["global_batch"] == 4
    assert res["k4_train"]["config"]["global_batch"] == 2 and res["k4_train"]["config"]["parallelism"] == "dp2"
    assert res["fp32_train"]["config"]["global_batch"] == 2 and res["fp32_train"]["dtype"] == "f32"
    for leg in ("k4_train", "fp32_train", "fp32_infer"):
        assert "roofline" in res[leg] and "error" not in res[leg], res[leg]


def test_rccl_one_rank_fit_generator():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    port = str(29900 + os.getpid() % 90)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.join(ROOT, "tools", "rccl_world1.py")]
    env = dict(os.environ, CNNITMO_DIST_FORCE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("CNNITMO_DIST_BACKEND", None)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("bit-identical") == 2, r.stdout
    print(r.stdout.strip())
