"""Data-parallel rehearsal on ONE GPU: N ranks share device 0 over gloo
(CNNITMO_DEVICE=0, CNNITMO_DIST_BACKEND=gloo) and train through the PUBLIC path
the reference uses -- paired ImageDataGenerator streams zipped into
``Model.fit_generator`` (main.py:82-132) with ``distributed=True`` -- so the
rank-sharded generators, the bucketed all-reduce launched during backward, the
averaged BN moving statistics and the global epoch logs all run for real.

Checks (rank 0):
  * every rank ends with bit-identical parameters and moving statistics;
  * they equal a single-process replay that draws the UNSHARDED stream at the
    global batch size (batch * world), splits each global batch into the ranks'
    shares, runs each share with that rank's dropout seed from the same starting
    state, normalises each share's loss gradient by N/world frames as the DP path does,
    averages the moving statistics itself and applies RMSprop once: bit-identical (the
    same roundings matter: a bias feeding a BatchNormalization has a zero gradient up to
    rounding, and RMSprop's first step turns such residues into updates of up to
    lr*sqrt(10), so two orders of the same sum differ by 1e-6 in the parameters);
  * fp32, independently of the DP path's normalisation: the same shares by their own
    batch means, weighted by n_r/N (the 11-frame stream ends in a 3-frame global batch:
    shares 2 and 1), give the global batch mean's gradient to 1e-5 of its largest entry;
  * the epoch loss equals the sample-weighted mean of the replay's per-share losses.
  * ``Model.fit(x, y, batch_size=B, distributed=True)`` -- batch_size is PER RANK, as
    for the generators -- on 11 frames (global batches 4, 4, 3: shares 2+2, 2+2, 2+1)
    and on 9 frames (4, 4, then a 1-frame tail with fewer frames than ranks, dropped on
    every rank): the step count, identical replicas and the same single-process replay.

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
from cnn_itmo_amd import ops  # noqa: E402
from cnn_itmo_amd.datagen import ImageDataGenerator  # noqa: E402

H, W, B, STEPS, NFR = 64, 96, 2, 3, 11
AUG = dict(rescale=1. / 255, rotation_range=90, horizontal_flip=True, vertical_flip=True, zoom_range=0.2)


def frames():
    rng = np.random.default_rng(42)
    x = rng.integers(0, 256, size=(NFR, H, W, 3), dtype=np.uint8)
    y = rng.integers(0, 256, size=(NFR, H, W, 3), dtype=np.uint8)
    return x, y


def model(dtype):
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        return C.U_net(input_size=(H, W, 3), dtype=dtype, seed=3, verbose=False)


def main():
    rank, world, local = D.init_from_env()
    torch.cuda.set_device(local)
    dtype = os.environ.get("DTYPE", "float32")
    X, Y = frames()
    m = model(dtype)
    if rank != 0:  # rank 0's initial state must win (DDP broadcast)
        m.set_named_weights({k: v + 0.25 for k, v in m.named_weights().items() if k.endswith("/kernel")})
    m.distribute(bucket_mb=0.5)  # several buckets, launched during backward
    gx = ImageDataGenerator(**AUG).flow(X, batch_size=B, seed=1)  # sharded over the group
    gy = ImageDataGenerator(**AUG).flow(Y, batch_size=B, seed=1)
    assert (gx.rank, gx.world) == (rank, world)
    hist = m.fit_generator(zip(gx, gy), steps_per_epoch=STEPS, epochs=1, verbose=0)
    eng = m.engine
    torch.cuda.synchronize()
    p = eng.params.cpu().numpy()
    bufs = eng.bufs.cpu().numpy()
    digest = hashlib.sha256(p.tobytes() + bufs.tobytes()).hexdigest()
    out = [None] * world
    dist.all_gather_object(out, digest)
    if rank == 0:
        assert len(set(out)) == 1, f"ranks diverged: {out}"
        # single-process replay at the global batch size
        rx = ImageDataGenerator(**AUG).flow(X, batch_size=B * world, seed=1, world=1)
        ry = ImageDataGenerator(**AUG).flow(Y, batch_size=B * world, seed=1, world=1)
        q, qb, lmean = replay(dtype, world, [(next(rx), next(ry)) for _ in range(STEPS)])
        err = float(np.abs(p - q).max())
        berr = float(np.abs(bufs - qb).max())
        lerr = abs(hist.history["loss"][0] - lmean)
        print(f"dp rehearsal: {world} ranks identical ({out[0][:12]}), max |dp - replay| params = {err:.3e}, "
              f"moving stats = {berr:.3e}, epoch loss {hist.history['loss'][0]:.6f} vs {lmean:.6f}")
        assert err == 0.0, err
        assert berr == 0.0, berr
        assert lerr <= 1e-6 * max(1.0, lmean), lerr
    dist.barrier()
    for nfr in (NFR, 9):
        fit_phase(dtype, rank, world, nfr)


def replay(dtype, world, batches):
    """Single process: each global batch split into the ranks' shares (np.array_split),
    each share run with that rank's dropout seed from the same state and its loss
    gradient normalised by N/world frames, moving statistics averaged, one RMSprop step
    per global batch.  fp32: each share is also run by its own batch mean and weighted by
    n_r/N, and that sum must be the same gradient (to 1e-5 of its largest entry).
    -> (params, moving stats, sample-weighted mean loss)."""
    r = model(dtype)
    e2 = r._engine()
    lsum, nsum = 0.0, 0
    for s, (xb, yb) in enumerate(batches):
        parts = [np.array_split(np.arange(len(xb)), world)[k] for k in range(world)]
        acc = torch.zeros_like(e2.grads)
        ind = torch.zeros_like(e2.grads)
        b0 = e2.bufs.clone()
        bacc = torch.zeros_like(e2.bufs)
        runs = 0
        for k, ix in enumerate(parts):
            ix = torch.as_tensor(ix, device=xb.device)
            if dtype == "float32":
                e2.bufs.copy_(b0)
                e2.train_step(xb[ix], yb[ix], seed=s * world + k, apply=False)
                ind += e2.grads * (len(ix) / len(xb))  # the global batch mean's gradient
                runs += 1
            e2.bufs.copy_(b0)
            la = e2.train_step(xb[ix], yb[ix], seed=s * world + k, apply=False, grad_frames=len(xb) / world)
            acc += e2.grads
            runs += 1
            lsum += float(la[0]) * len(ix)
            nsum += len(ix)
            bacc += e2.bufs
        if dtype == "float32":
            gerr = float((acc / world - ind).abs().max())
            assert gerr <= 1e-5 * float(ind.abs().max()), (gerr, float(ind.abs().max()))
        e2.step -= runs - 1
        e2.bufs.copy_(bacc * (1.0 / world))
        ops.rmsprop(e2.params, acc, e2.accum, 1e-3, 0.9, 1e-7, 1.0 / world)
        e2.weights_dirty = True
    torch.cuda.synchronize()
    return e2.params.cpu().numpy(), e2.bufs.cpu().numpy(), lsum / nsum


def fit_phase(dtype, rank, world, nfr):
    """Model.fit under DP: batch_size is per rank (global batch B * world); a global
    batch with fewer frames than ranks is dropped on every rank."""
    X, Y = frames()
    X = (X[:nfr] / 255.0).astype(np.float32)
    Y = (Y[:nfr] / 255.0).astype(np.float32)
    m = model(dtype)
    if rank != 0:
        m.set_named_weights({k: v + 0.25 for k, v in m.named_weights().items() if k.endswith("/kernel")})
    hist = m.fit(X, Y, batch_size=B, epochs=1, shuffle=False, verbose=0, distributed=True)
    gb = B * world
    blocks = [np.arange(i, min(i + gb, nfr)) for i in range(0, nfr, gb)]
    blocks = [b for b in blocks if len(b) >= world]
    eng = m.engine
    assert eng.step == len(blocks), (eng.step, len(blocks))
    torch.cuda.synchronize()
    p, bufs = eng.params.cpu().numpy(), eng.bufs.cpu().numpy()
    out = [None] * world
    dist.all_gather_object(out, hashlib.sha256(p.tobytes() + bufs.tobytes()).hexdigest())
    if rank == 0:
        assert len(set(out)) == 1, f"Model.fit ranks diverged: {out}"
        dev = eng.params.device
        q, qb, lmean = replay(dtype, world, [(torch.as_tensor(X[b], device=dev), torch.as_tensor(Y[b], device=dev))
                                             for b in blocks])
        err = float(np.abs(p - q).max())
        lerr = abs(hist.history["loss"][0] - lmean)
        print(f"Model.fit {nfr} frames: {len(blocks)} steps (global batches {[len(b) for b in blocks]}), "
              f"ranks identical, max |dp - replay| params = {err:.3e}, epoch loss {hist.history['loss'][0]:.6f} "
              f"vs {lmean:.6f}")
        assert err == 0.0, err
        assert float(np.abs(bufs - qb).max()) == 0.0
        assert lerr <= 1e-6 * max(1.0, lmean), lerr
    dist.barrier()


if __name__ == "__main__":
    main()
