"""Data-parallel rehearsal on ONE GPU: N ranks share device 0 over gloo
(CNNITMO_DEVICE=0, CNNITMO_DIST_BACKEND=gloo) and run the real engine + the
bucketed all-reduce (cnn_itmo_amd/dist.py) with different data per rank.  After
K steps every rank must hold bit-identical parameters, and they must equal a
single-process replay that averages the ranks' gradients itself.

  CNNITMO_DEVICE=0 CNNITMO_DIST_BACKEND=gloo python -m torch.distributed.run \\
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/dp_rehearsal.py
"""
import contextlib
import hashlib
import io
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cnn_itmo_amd as C  # noqa: E402
from cnn_itmo_amd import dist as D  # noqa: E402

H, W, B, STEPS = 64, 96, 2, 3


def batch(rank, step):
    g = torch.Generator(device="cuda")
    g.manual_seed(100 + 7 * rank + 1000 * step)
    x = torch.rand(B, H, W, 3, generator=g, device="cuda")
    t = torch.rand(B, H, W, 3, generator=g, device="cuda")
    return x, t


def model(dtype):
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        return C.U_net(input_size=(H, W, 3), dtype=dtype, seed=3, verbose=False)


def main():
    rank, world, local = D.init_from_env()
    torch.cuda.set_device(local)
    dtype = os.environ.get("DTYPE", "float32")
    m = model(dtype)
    eng = m._engine()
    b = D.attach(eng, bucket_mb=0.5)  # several buckets, launched during backward
    for s in range(STEPS):
        x, t = batch(rank, s)
        eng.train_step(x, t, seed=s, sync=b.finish, grad_scale=b.grad_scale)
    torch.cuda.synchronize()
    p = eng.params.cpu().numpy()
    digest = hashlib.sha256(p.tobytes()).hexdigest()
    out = [None] * world
    dist.all_gather_object(out, digest)
    if rank == 0:
        assert len(set(out)) == 1, f"ranks diverged: {out}"
        # single-process replay: per-rank gradients averaged by hand, same RMSprop
        r = model(dtype)
        e2 = r._engine()
        for s in range(STEPS):
            acc = torch.zeros_like(e2.grads)
            for k in range(world):
                x, t = batch(k, s)
                e2.train_step(x, t, seed=s, apply=False)
                acc += e2.grads
            e2.step -= world - 1
            from cnn_itmo_amd import ops
            ops.rmsprop(e2.params, acc, e2.accum, 1e-3, 0.9, 1e-7, 1.0 / world)
            e2.weights_dirty = True
        torch.cuda.synchronize()
        q = e2.params.cpu().numpy()
        err = float(np.abs(p - q).max())
        print(f"dp rehearsal: {world} ranks identical ({out[0][:12]}), max |dp - replay| = {err:.3e}")
        assert err <= 1e-6 * max(1.0, float(np.abs(q).max())), err
    dist.barrier()


if __name__ == "__main__":
    main()
