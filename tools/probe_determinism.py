"""Run-to-run determinism of one training step (GPU).

    DTYPE=float32 python tools/probe_determinism.py [H W N]

Builds the U-Net, runs train_step(apply=False) twice on the same frames with the same
dropout seed and compares the gradient buffers bit for bit, per parameter tensor.  Every
reduction in the library is fixed-order (slab reductions, partial-sum rows), so any
difference names a kernel that reads something it did not write (or races).
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cnn_itmo_amd as C  # noqa: E402


def main():
    dtype = os.environ.get("DTYPE", "float32")
    h, w, n = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (64, 96, 2)
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(h, w, 3), dtype=dtype, seed=3, verbose=False)
    e = m._engine()
    rng = np.random.default_rng(5)
    x = torch.tensor(rng.random((n, h, w, 3), dtype=np.float32)).cuda()
    t = torch.tensor(rng.random((n, h, w, 3), dtype=np.float32)).cuda()
    gs, ls = [], []
    for rep in range(3):
        la = e.train_step(x, t, seed=7, apply=False)
        torch.cuda.synchronize()
        gs.append(e.grads.clone())
        ls.append(la.cpu().numpy().tolist())
    bad = []
    for name, (off, shp) in e.pslices.items():
        k = int(np.prod(shp))
        for rep in (1, 2):
            d = (gs[rep][off:off + k] - gs[0][off:off + k]).abs().max().item()
            if d != 0.0:
                bad.append((name, rep, d))
    print(f"{dtype} {n}x{h}x{w}: losses {ls}")
    print("deterministic" if not bad else f"{len(bad)} differing tensors:")
    for name, rep, d in bad[:40]:
        print(f"  {name:40s} rep {rep}: max |diff| {d:.3e}")


if __name__ == "__main__":
    main()
