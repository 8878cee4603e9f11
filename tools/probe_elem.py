"""HIP-event timings of the level-0 HBM passes at the bench shape (GPU box):
head fwd+bwd (g3) and the g3 BN-backward apply.  python tools/probe_elem.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnn_itmo_amd import ops  # noqa: E402


def timeit(f, iters=6):
    ts = []
    for _ in range(iters):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts[1:])[len(ts[1:]) // 2]


def main():
    dt, T = ops.DTYPES["bfloat16"]
    B, H, Hv, W, C = 32, 1088, 1080, 1920, 64
    P = B * H * W
    x = ops.new_view(B, H, W, C, T)
    x.buf.normal_()
    wt = torch.randn(3 * C, device="cuda") * 0.1
    b = torch.zeros(3, device="cuda")
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.1
    target = torch.rand(B * Hv * W * 3, device="cuda")
    g3 = torch.empty(P * 3, device="cuda")
    rows = ops.head_rows(P)
    part = torch.empty(rows * (5 + 3 * C), device="cuda")
    t = timeit(lambda: ops.head_fwd_bwd_g3(dt, x, Hv, wt, b, target, g3, part, aff=(sc, sh)))
    gb = (P * C * 2 + B * Hv * W * 12 + P * 12) / 1e9
    print(f"head_fwd_bwd_g3   {t:7.3f} ms  {gb / t:6.2f} TB/s (algorithmic {gb:.1f} GB)", flush=True)
    y = torch.empty_like(x.buf)
    t = timeit(lambda: y.copy_(x.buf))
    gb = 2 * P * C * 2 / 1e9
    print(f"torch copy (ref)  {t:7.3f} ms  {gb / t:6.2f} TB/s (algorithmic {gb:.1f} GB)", flush=True)
    del y
    coef = torch.rand(3 * C, device="cuda")
    dz = torch.empty(P * C, dtype=T, device="cuda")
    prow = ops.query("cnnitmo_bn_bwd_rows", P, C)
    part2 = torch.empty(prow * C * 2, device="cuda")
    t = timeit(lambda: ops.bn_bwd_apply_g3(dt, g3, wt, x, C, P, coef, dz, part2))
    gb = (P * 12 + P * C * 2 * 2) / 1e9
    print(f"bn_bwd_apply_g3   {t:7.3f} ms  {gb / t:6.2f} TB/s (algorithmic {gb:.1f} GB)", flush=True)


if __name__ == "__main__":
    main()
