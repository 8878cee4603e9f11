"""The fp64 (and fp32, and bf16-storage) numpy oracle of ONE training step at the benchmarked
frame size (test infrastructure, CPU only: tests/golden/make_train1080.py reduces its outputs to
the committed fixture tests/golden/train1080.npz, which tests/test_gpu_train1080.py reads; the
GPU tests never run this script).

    python tools/train1080_oracle.py --out /tmp/o.npz [--dtype float64|float32|bf16store]

bf16store: fp64 arithmetic with every stored tensor rounded to bfloat16 (UNetRef(store=
R.round_bf16), the emulation test_gpu_model.py's 128x128 bf16 test uses): the noise floor a
bf16-storage implementation with wide accumulation is held to.

Input: the 12 reference SDR frames tiled into one real-content 1080x1920 frame
(tests/golden/make_golden.mosaic1080), zero-padded to 1088 rows as U_net(pad=True) pads
it; weights: sdr1080.npz's seeded U-Net parameters; target: a seeded tone curve of the
input; dropout seed 5.  The loss covers the 1080 valid rows only (oracle
UNetRef.backward(valid_rows=...)).  Saves the loss, the metric, all 74 gradients and
the Keras moving statistics after the step (bn_moving_update of the batch statistics).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLD)

from oracle import unet_ref as R  # noqa: E402

SEED = 5  # dropout seed of the step
H, W, HP = 1080, 1920, 1088


def inputs():
    """(params, x [1,1080,1920,3], target [1,1080,1920,3]) of the 1080p training check."""
    from PIL import Image
    from make_golden import mosaic1080, seeded_unet_params
    z = np.load(os.path.join(GOLD, "sdr1080.npz"), allow_pickle=False)
    names = [str(n) for n in z["names"]]
    frames = []
    for nm in names:
        with Image.open(os.path.join(GOLD, "sdr512", nm)) as im:
            frames.append(np.asarray(im.convert("RGB")))
    P = seeded_unet_params(*z["w_seed"].tolist())
    x = R.png_to_input(mosaic1080(frames))[None]
    rng = np.random.default_rng(1080)
    t = np.clip(x ** 2.2 * 1.2 + rng.uniform(-0.02, 0.02, x.shape), 0.0, 1.0)
    return P, x, t


def run(dtype, out, store=None):
    P, x, t = inputs()
    xp = np.zeros((1, HP, W, 3))
    xp[:, :H] = x
    net = R.UNetRef(P, dtype, store=store)
    t0 = time.perf_counter()
    net.forward(xp.astype(dtype), training=True, seed=SEED)
    t1 = time.perf_counter()
    loss, acc, grads = net.backward(t.astype(dtype), valid_rows=H)
    t2 = time.perf_counter()
    mov = {}
    for name, entry in net.cache.items():
        if isinstance(entry, dict) and entry.get("stats"):
            bn = entry["bn"]
            m, v, n = entry["stats"][0]
            mm, mv = R.bn_moving_update(net.P[bn + "/moving_mean"], net.P[bn + "/moving_variance"], m, v, n)
            mov[bn + "/moving_mean"], mov[bn + "/moving_variance"] = mm, mv
    d = {"loss": np.array(loss), "acc": np.array(acc), "seconds": np.array([t1 - t0, t2 - t1])}
    d.update({"g/" + k: np.asarray(v, np.float64) for k, v in grads.items()})
    d.update({"m/" + k: np.asarray(v, np.float64) for k, v in mov.items()})
    tmp = out + ".tmp.npz"
    np.savez(tmp, **d)
    os.replace(tmp, out)
    print(f"[train1080_oracle] {np.dtype(dtype).name}{' bf16 storage' if store else ''}: fwd {t1 - t0:.1f} s, bwd {t2 - t1:.1f} s, loss {loss:.9f}",
          file=sys.stderr, flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--dtype", default="float64", choices=["float64", "float32", "bf16store"])
    a = ap.parse_args()
    if a.dtype == "bf16store":
        run(np.float64, a.out, store=R.round_bf16)
    else:
        run(np.float64 if a.dtype == "float64" else np.float32, a.out)
