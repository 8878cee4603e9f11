"""Tiled vs whole-frame inference on the GPU: equality and time (GPU box).

    python tools/tiled_probe.py [--h 2160] [--w 3840] [--n 2] [--tile 1024,1024]

Prints, per dtype, the max |tiled - full| and the fraction of bit-equal outputs, and
the wall time of each path (HIP-synchronised, second of two runs)."""
import argparse
import contextlib
import io
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cnn_itmo_amd as C  # noqa: E402
from cnn_itmo_amd.tiled import predict_tiled  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--n", type=int, default=2)
    ap.add_argument("--tile", default="1024,1024")
    a = ap.parse_args()
    tile = tuple(int(v) for v in a.tile.split(","))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randint(0, 256, (a.n, a.h, a.w, 3), generator=g, device="cuda").float() / 255
    for dt in ("float32", "bfloat16"):
        C.clear_session()
        with contextlib.redirect_stdout(io.StringIO()):
            m = C.U_net(input_size=(a.h, a.w, 3), pad=True, dtype=dt, seed=2, verbose=False)
        eng = m._engine()
        res = {}
        for name, fn in (("full", lambda: eng.predict(x)),
                         ("tiled", lambda: predict_tiled(m, x, tile, batch_size=8, cache=cache))):
            cache = {}
            for _ in range(2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                y = fn()
                torch.cuda.synchronize()
                dtm = time.perf_counter() - t0
            res[name] = (y, dtm)
            print(f"{dt:9s} {name:5s} {a.n}x{a.h}x{a.w}: {dtm * 1e3:8.1f} ms  peak {torch.cuda.max_memory_allocated() / 2**30:6.1f} GiB",
                  flush=True)
            torch.cuda.reset_peak_memory_stats()
        d = (res["tiled"][0] - res["full"][0]).abs()
        print(f"{dt:9s} max|tiled-full| {float(d.max()):.3e}  bit-equal {float((d == 0).float().mean()):.6f}  "
              f"tile {tile}", flush=True)
        del eng, m, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
