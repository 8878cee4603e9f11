"""First-layer conv (conv_c3_fwd) at the bench shape: time per launch (HIP events,
median of 10) and a checksum of the output and BN partial sums (GPU box):
    python tools/probe_c3.py [--batch 32]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnn_itmo_amd import _lib as L, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--ld", type=int, default=32, help="output row pitch (32: dense conv1 as the engine stores it)")
    a = ap.parse_args()
    n, hv, h, w = a.batch, 1080, 1088, 1920
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand(n, hv, w, 3, generator=g, device="cuda")
    wt = (torch.randn(32 * 32, generator=g, device="cuda") * 0.2).to(torch.bfloat16)
    bias = torch.randn(32, generator=g, device="cuda") * 0.1
    out = ops.View(torch.zeros(n * h * w * a.ld, dtype=torch.bfloat16, device="cuda"), n, h, w, 32, a.ld, 0)
    rows = ops.query("cnnitmo_conv_c3_stat_rows", n, h, w)
    st = torch.zeros(rows * 64, device="cuda")
    f = lambda: ops.conv_c3_fwd(L.BF16, x, n, hv, h, w, wt, bias, out, L.RELU | L.STATS, None, st)  # noqa: E731
    f()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    y = out.tensor().float()
    gb = (n * hv * w * 12 + n * h * w * 64) / 1e9
    ms = float(np.median(ts))
    print(f"conv_c3_fwd {n}x{h}x{w}: {ms:.3f} ms  {gb / ms:.2f} TB/s (12 B in + 64 B out per pixel)  "
          f"sum(out) {float(y.double().sum()):.6e}  sum(stats) {float(st.view(rows, 2, 32).double().sum(0).sum()):.6e}")
    dz = (torch.randn(n * h * w * 32, generator=g, device="cuda") * 0.1).to(torch.bfloat16)
    dw = torch.empty(32 * 27, device="cuda")
    fw = lambda: ops.conv_c3_wgrad(L.BF16, x, n, hv, h, w, dz, dw)  # noqa: E731
    fw()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fw()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    print(f"conv_c3_wgrad {n}x{h}x{w}: {ms:.3f} ms  {gb / ms:.2f} TB/s (12 B + 64 B read per pixel)  "
          f"sum(dw) {float(dw.double().sum()):.6e}  sum|dw| {float(dw.double().abs().sum()):.6e}")


if __name__ == "__main__":
    main()
