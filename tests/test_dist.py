"""Data-parallel path on CPU (gloo, world size 2): each rank computes its shard's
gradients (the numpy oracle stands in for the GPU engine here), writes them into
the engine's flat gradient layout, and runs the real GradBucketer
(cnn_itmo_amd/dist.py) in backward order.  The averaged result must equal the
oracle's full-batch gradient with per-replica BatchNorm (bn groups = world)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bucket_mb, errq):
    try:
        import sys
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        from cnn_itmo_amd import dist as D
        r, w, _ = D.init_from_env(backend="gloo")
        assert (r, w) == (rank, world)
        import cnn_itmo_amd as C
        from cnn_itmo_amd.engine import compile_graph, layout_params
        from oracle import unet_ref as R
        C.clear_session()
        m = C.U_net(input_size=(32, 32, 3), verbose=False)
        stages = compile_graph(m)
        ps, _, goff, n, _ = layout_params(stages)
        P = R.init_unet_params(1)
        rng = np.random.default_rng(0)
        x = rng.uniform(size=(2 * world, 32, 32, 3))
        t = rng.uniform(size=x.shape)
        seeds = [100 + k for k in range(world)]
        sl = slice(2 * rank, 2 * rank + 2)
        net = R.UNetRef(P)
        net.forward(x[sl], training=True, seed=seeds[rank])
        _, _, g = net.backward(t[sl])
        flat = torch.zeros(n, dtype=torch.float64)
        b = D.GradBucketer(flat, goff[::-1], bucket_mb=bucket_mb)
        assert len(b.buckets) >= (2 if bucket_mb < 1 else 1)
        # emulate the engine: write each stage's grads, then fire the hook (backward order)
        for i in range(len(stages) - 1, -1, -1):
            for k, shp in stages[i].params:
                off, _ = ps[k]
                flat[off:off + g[k].size] = torch.from_numpy(g[k].reshape(-1))
            if stages[i].params:
                b.hook(*goff[i])
        b.finish()
        avg = flat * b.grad_scale
        full = R.UNetRef(P)
        full.forward(x, training=True, groups=world, drop_seeds=seeds)
        _, _, gf = full.backward(t)
        for k, (off, shp) in ps.items():
            got = avg[off:off + int(np.prod(shp))].numpy().reshape(gf[k].shape)
            np.testing.assert_allclose(got, gf[k], rtol=1e-9, atol=1e-14, err_msg=k)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface to the parent
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


@pytest.mark.parametrize("bucket_mb", [0.25, 64.0])
def test_dp_gradient_allreduce_equals_full_batch(bucket_mb):
    world = 2
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_make_buckets():
    from cnn_itmo_amd.dist import make_buckets
    r = [(0, 10), (10, 10), (10, 50), (50, 55), (55, 200)]
    assert make_buckets(r, 40) == [(0, 50), (50, 200)]
    assert make_buckets(r, 1000) == [(0, 200)]
    assert make_buckets(r, 1) == [(0, 10), (10, 50), (50, 55), (55, 200)]
