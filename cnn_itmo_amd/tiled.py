"""Spatially tiled inference: SURVEY 8e / BASELINE configs[4] "spatially tiled
activations" -- tiles on a 16-aligned grid with >= 96-px halos, exact for inference.

The U-Net (model.py:204-278) is fully convolutional and, in inference, every BN is
a per-channel affine map, so an output pixel depends only on the input pixels in
its receptive field: 170 px wide (3x3 convs at strides 1..16 plus the 2x2 pools;
the transposed convs add none), i.e. at most 93 px to either side of a pixel once
the 16-pixel pooling alignment is counted.  A frame is therefore cut into tiles on
a 16-aligned grid; each tile runs through the same network built for a fixed
WINDOW = tile + 2 x halo (a multiple of 16), and only the tile's interior is kept.
Windows are shifted inward at the frame's edges instead of being zero-padded: a
window edge then either lies >= halo pixels from every kept pixel or IS the frame's
edge, where the full-frame network's own zero padding applies, so the result equals
the full-frame prediction (bit-identical here: every kernel computes a pixel's dot
products in an order that does not depend on where the pixel sits in its launch;
tests/test_gpu_tiled.py).

This bounds the activation memory by the window, not the frame (8K frames or
large batches of 4K frames), at the cost of recomputing the halos:
(tile + 2 halo)^2 / tile^2 of the work, 1.41x for 1024-px tiles.
"""
from __future__ import annotations

import numpy as np

HALO = 96  # >= 93 (see above), a multiple of 16


def _round16(v):
    return -(-int(v) // 16) * 16


def windows(size, tile, halo=HALO):
    """[(s, a, b)]: window rows [s, s + win) and the kept rows [a, b) of a dimension of
    ``size`` (a multiple of 16) cut into ``tile``-row tiles; win = min(tile + 2 halo, size)."""
    if size % 16 or tile % 16 or halo % 16 or tile <= 0:
        raise ValueError(f"size {size}, tile {tile}, halo {halo}: all must be multiples of 16")
    win = min(tile + 2 * halo, size)
    out = []
    for a in range(0, size, tile):
        b = min(a + tile, size)
        s = min(max(a - halo, 0), size - win)
        out.append((s, a, b))
    return win, out


def predict_tiled(model, x, tile=(1024, 1024), halo=HALO, batch_size=8, cache=None):
    """Inference of ``model`` (a U-Net of any input size; same weights) on frames x
    [N, H, W, 3] float (host array or CUDA tensor) through windows of (tile + 2 halo);
    returns float32 [N, H, W, 3] (a host array for host input, else a CUDA tensor).
    H, W are zero-padded to multiples of 16 like the full-frame predict."""
    import torch
    from .predict import model_for_size
    host = not isinstance(x, torch.Tensor)
    xt = torch.as_tensor(np.asarray(x, dtype=np.float32)) if host else x.float()
    xt = xt.cuda()
    if xt.ndim != 4 or xt.shape[3] != 3:
        raise ValueError(f"expected [N, H, W, 3] frames, got {tuple(xt.shape)}")
    n, h, w, _ = xt.shape
    H, W = _round16(h), _round16(w)
    if (H, W) != (h, w):
        xp = torch.zeros(n, H, W, 3, device=xt.device, dtype=torch.float32)
        xp[:, :h, :w] = xt
        xt = xp
    th, tw = int(tile[0]), int(tile[1])
    wh, rows = windows(H, th, halo)
    ww, cols = windows(W, tw, halo)
    m = model_for_size(model, wh, ww, cache)
    eng = m._engine()
    out = torch.empty(n, H, W, 3, device=xt.device, dtype=torch.float32)
    jobs = [(i, r, c) for i in range(n) for r in rows for c in cols]
    for j in range(0, len(jobs), batch_size):
        part = jobs[j:j + batch_size]
        xb = torch.stack([xt[i, r[0]:r[0] + wh, c[0]:c[0] + ww] for i, r, c in part])
        yb = eng.predict(xb)
        for k, (i, (s, a, b), (sc, ac, bc)) in enumerate(part):
            out[i, a:b, ac:bc] = yb[k, a - s:b - s, ac - sc:bc - sc]
    out = out[:, :h, :w]
    return out.cpu().numpy() if host else out
