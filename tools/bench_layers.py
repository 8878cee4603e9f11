"""Per-layer conv microbenchmark on the U-Net's real shapes (1088x1920, batch B).

    python tools/bench_layers.py [--batch 32] [--dtype bfloat16] [--ops fwd,dgrad,wgrad] [--iters 5]

Times each conv op of each layer with HIP events (median of iters) and prints
TFLOP/s (algorithmic 2*MAC) and the share of total conv time.
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnn_itmo_amd import ops  # noqa: E402

H0, W0 = 1088, 1920
# name, kind, level (spatial /2^level), cin, cout
LAYERS = [
    ("enc1b", "c3", 0, 32, 32), ("enc2a", "c3", 1, 32, 64), ("enc2b", "c3", 1, 64, 64),
    ("enc3a", "c3", 2, 64, 128), ("enc3b", "c3", 2, 128, 128), ("enc4a", "c3", 3, 128, 256),
    ("enc4b", "c3", 3, 256, 256), ("crossa", "c3", 4, 256, 512), ("crossb", "c3", 4, 512, 512),
    ("up6", "t2", 4, 512, 512), ("dec6", "c3", 3, 768, 512), ("up7", "t2", 3, 512, 256),
    ("dec7", "c3", 2, 384, 256), ("up8", "t2", 2, 256, 128), ("dec8", "c3", 1, 192, 128),
    ("up9", "t2", 1, 128, 64), ("dec9", "c3", 0, 96, 64),
    # conv9's input gradient for its up9 columns alone (the split launch, engine._split_fused:
    # dz 64 channels -> the 64 columns of up9), as a 64 -> 64 shape; not a layer of its own
    ("dec9up", "c3", 0, 64, 64),
]


def timeit(fn, iters):
    fn()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--layers", default="")
    a = ap.parse_args()
    dt, T = ops.DTYPES[a.dtype]
    B = a.batch
    want = set(a.ops.split(","))
    sel = set(a.layers.split(",")) if a.layers else None
    rows = []
    for name, kind, lvl, cin, cout in LAYERS:
        if sel and name not in sel:
            continue
        h, w = H0 >> lvl, W0 >> lvl
        if kind == "t2":
            hi, wi = h, w  # input grid of the tconv
            x = ops.new_view(B, hi, wi, cin, T)
            x.buf.uniform_(-1, 1)
            k = torch.randn(4 * cout * cin, device="cuda").to(T) * 0.05
            kT = k.clone()
            bias = torch.zeros(cout, device="cuda", dtype=torch.float32)
            out = ops.new_view(B, 2 * hi, 2 * wi, cout, T)
            fl = 2.0 * B * hi * wi * 4 * cout * cin
            if "fwd" in want:  # ReLU + BN partial sums, as in the training step
                st = torch.empty(ops.tconv_stat_rows(dt, B, hi, wi, cin, cout) * 2 * 4 * cout, device="cuda")
                rows.append((name, "fwd", fl, timeit(lambda: ops.tconv_fwd(dt, x, k, bias, out, 1 | 2, stats=st), a.iters)))
            if "dgrad" in want:
                dx = torch.empty(B * hi * wi * cin, dtype=T, device="cuda")
                rows.append((name, "dgrad", fl, timeit(lambda: ops.tconv_dgrad(dt, out.buf, B, hi, wi, cout, kT, cin, dx), a.iters)))
            if "wgrad" in want:
                dk = torch.empty(4 * cout * cin, device="cuda", dtype=torch.float32)
                rows.append((name, "wgrad", fl, timeit(lambda: ops.tconv_wgrad(dt, x, out.buf, cout, dk), a.iters)))
            del x, out
        else:
            x = ops.new_view(B, h, w, cin, T)
            x.buf.uniform_(-1, 1)
            wt = torch.randn(cout * 9 * cin, device="cuda").to(T) * 0.05
            bias = torch.zeros(cout, device="cuda", dtype=torch.float32)
            out = ops.new_view(B, h, w, cout, T)
            fl = 2.0 * B * h * w * cout * 9 * cin
            if "fwd" in want:
                rows.append((name, "fwd", fl, timeit(lambda: ops.conv3x3_fwd(dt, x, wt, bias, out, 1), a.iters)))
            if "dgrad" in want:
                dx = ops.new_view(B, h, w, cin, T)
                rows.append((name, "dgrad", fl, timeit(lambda: ops.conv3x3_dgrad(dt, out.buf, B, h, w, cout, wt, cin, dx), a.iters)))
            if "dgradbn" in want and (name.startswith("dec") or lvl == 0):
                # decoder dgrad with the up-path producer's BN backward fused (engine: concat
                # [skip, up], up = the tconv output at channels [cin - cout, cin), parity sums);
                # a level-0 conv whose whole input is the previous conv's BN output: [0, cin)
                par = name.startswith("dec") and name != "dec9up"
                c0, c1 = (cin - cout, cin) if par else (0, cin)
                dx = ops.new_view(B, h, w, cin, T)
                r = ops.View(x.buf, B, h, w, c1 - c0, cin, c0)
                coef = torch.rand(3 * (c1 - c0), device="cuda")
                rows_ = ops.conv3x3_dgrad_bn_rows(dt, B, h, w, cout, cin, c0, c1)
                dzp = torch.empty(B * h * w * (c1 - c0), dtype=T, device="cuda")
                pp = torch.empty(rows_ * 4 * (c1 - c0), device="cuda")
                rows.append((name, "dgradbn", fl, timeit(lambda: ops.conv3x3_dgrad_bn(
                    dt, out.buf, B, h, w, cout, wt, cin, dx, c0, c1, coef, r, dzp, pp, par), a.iters)))
            if "wgrad" in want:
                dw = torch.empty(cout * 9 * cin, device="cuda", dtype=torch.float32)
                rows.append((name, "wgrad", fl, timeit(lambda: ops.conv_wgrad(dt, 9, x, out.buf, cout, dw), a.iters)))
            if "wgradcat" in want and cin == 96:  # dec9's [conv1 32 | up9 64] read from its two members
                x1, x2 = ops.new_view(B, h, w, 32, T), ops.new_view(B, h, w, 64, T)
                x1.buf.uniform_(-1, 1)
                x2.buf.uniform_(-1, 1)
                dw = torch.empty(cout * 9 * cin, device="cuda", dtype=torch.float32)
                rows.append((name, "wgcat", fl, timeit(lambda: ops.conv_wgrad_cat(dt, x1, x2, out.buf, cout, dw), a.iters)))
                del x1, x2
            del x, out
        torch.cuda.empty_cache()
    tot = sum(r[3] for r in rows)
    for name, op, fl, ms in rows:
        print(f"{name:7s} {op:6s} {ms:8.2f} ms {fl / ms / 1e9:8.1f} TFLOP/s  {ms / tot:6.1%}")
    tfl = sum(r[2] for r in rows)
    print(f"TOTAL   {tot:8.2f} ms {tfl / tot / 1e9:8.1f} TFLOP/s")


if __name__ == "__main__":
    main()
