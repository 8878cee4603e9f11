"""Spatially tiled inference (cnn_itmo_amd/tiled.py): the window plan, and -- on the
fp64 oracle, so without a GPU -- that cutting a frame into 16-aligned tiles with
96-px halos reproduces the full-frame forward (model.py:204-278 in inference mode),
while a too-small halo does not (the check is sensitive)."""
import numpy as np
import pytest

from cnn_itmo_amd.tiled import HALO, windows
from oracle import unet_ref as R


@pytest.mark.parametrize("size,tile", [(16, 16), (64, 32), (320, 64), (2160, 512), (1088, 1024), (3840, 1024),
                                       (4320, 256), (400, 128)])
def test_window_plan(size, tile):
    win, plan = windows(size, tile)
    assert win == min(tile + 2 * HALO, size) and win % 16 == 0
    covered = np.zeros(size, int)
    for s, a, b in plan:
        assert s % 16 == 0 and 0 <= s and s + win <= size  # windows lie inside the frame
        assert s <= a < b <= s + win
        covered[a:b] += 1
        # every kept row is >= HALO from a window edge unless that edge is the frame's
        assert s == 0 or a - s >= HALO
        assert s + win == size or s + win - b >= HALO
    assert (covered == 1).all()  # the kept rows partition the frame


def test_window_plan_rejects():
    with pytest.raises(ValueError):
        windows(100, 32)
    with pytest.raises(ValueError):
        windows(320, 40)


def _params(seed):
    P = R.init_unet_params(seed)
    rng = np.random.default_rng(seed + 1)
    for k in P:  # non-trivial inference BN (moving statistics, affine) and biases
        if k.endswith("moving_mean") or k.endswith("beta") or k.endswith("/bias"):
            P[k] = rng.normal(0, 0.1, P[k].shape)
        elif k.endswith("moving_variance") or k.endswith("gamma"):
            P[k] = rng.uniform(0.5, 1.5, P[k].shape)
    return P


def _tiled_oracle(net, x, tile, halo):
    n, H, W, _ = x.shape
    wh, rows = windows(H, tile[0], halo)
    ww, cols = windows(W, tile[1], halo)
    out = np.empty(x.shape)
    for s, a, b in rows:
        for sc, ac, bc in cols:
            y = net.forward(x[:, s:s + wh, sc:sc + ww], training=False)
            out[:, a:b, ac:bc] = y[:, a - s:b - s, ac - sc:bc - sc]
    return out


@pytest.mark.parametrize("shape,tile", [((320, 64), (64, 64)), ((64, 336), (64, 48))])
def test_tiled_oracle_equals_full_frame(shape, tile):
    """Tiles of 64 (48) with 96-px halos: 5 windows of 256 (240) along one dimension
    reproduce the full-frame fp64 forward to rounding; with 32-px halos they do not."""
    P = _params(3)
    net = R.UNetRef(P)
    rng = np.random.default_rng(5)
    x = rng.integers(0, 256, (1,) + shape + (3,)).astype(np.float64) / 255
    full = net.forward(x, training=False)
    tiled = _tiled_oracle(net, x, tile, HALO)
    assert float(np.abs(tiled - full).max()) <= 1e-12
    short = _tiled_oracle(net, x, tile, 32)
    assert float(np.abs(short - full).max()) > 1e-6
