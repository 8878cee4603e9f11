"""RCCL path on a one-GPU box: a one-rank ``nccl`` (= RCCL) process group with
CNNITMO_DIST_FORCE=1, so the DP path's collectives -- the state broadcast, the
bucketed gradient all-reduces launched during backward on RCCL's stream and the
moving-statistics all-reduce -- run for real (RCCL refuses two ranks on one GPU).
Trains through ``Model.fit_generator(..., distributed=True)`` (main.py:126-132) and
checks the parameters and moving statistics are bit-identical to the same training
without a process group (a one-rank sum is the identity, grad_scale 1).

  CNNITMO_DIST_FORCE=1 python -m torch.distributed.run --nproc-per-node 1 \\
      --master-addr 127.0.0.1 --master-port 29544 tools/rccl_world1.py
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cnn_itmo_amd as C  # noqa: E402
from cnn_itmo_amd import dist as D  # noqa: E402
from cnn_itmo_amd.datagen import ImageDataGenerator  # noqa: E402

H, W, B, STEPS = 64, 96, 2, 3


def train(distributed, dtype):
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(H, W, 3), dtype=dtype, seed=3, verbose=False)
    rng = np.random.default_rng(7)
    X = rng.integers(0, 256, size=(8, H, W, 3), dtype=np.uint8)
    Y = rng.integers(0, 256, size=(8, H, W, 3), dtype=np.uint8)
    if distributed:
        m.distribute(bucket_mb=0.5)  # several buckets, launched during backward
    gx = ImageDataGenerator(rescale=1. / 255, horizontal_flip=True).flow(X, batch_size=B, seed=1, world=1)
    gy = ImageDataGenerator(rescale=1. / 255, horizontal_flip=True).flow(Y, batch_size=B, seed=1, world=1)
    m.fit_generator(zip(gx, gy), steps_per_epoch=STEPS, epochs=1, verbose=0, distributed=distributed)
    torch.cuda.synchronize()
    return m


def main():
    assert os.environ.get("CNNITMO_DIST_FORCE") == "1"
    rank, world, local = D.init_from_env(backend="nccl")
    assert dist.is_initialized() and dist.get_backend() == "nccl" and world == 1
    torch.cuda.set_device(local)
    for dtype in ("float32", "bfloat16"):
        a = train(True, dtype)
        b = a._dp
        assert b is not None and b.collect and len(b.buckets) >= 2, "collectives not armed"
        pa, sa = a.engine.params.cpu().numpy(), a.engine.bufs.cpu().numpy()
        os.environ["CNNITMO_DIST_FORCE"] = "0"  # the reference run: no collectives
        r = train(False, dtype)
        os.environ["CNNITMO_DIST_FORCE"] = "1"
        assert r._dp is None
        pr, sr = r.engine.params.cpu().numpy(), r.engine.bufs.cpu().numpy()
        assert np.array_equal(pa, pr), float(np.abs(pa - pr).max())
        assert np.array_equal(sa, sr), float(np.abs(sa - sr).max())
        print(f"rccl world1 {dtype}: {len(b.buckets)} gradient buckets + moving stats all-reduced over RCCL, "
              f"params and moving stats bit-identical to the run without collectives")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
