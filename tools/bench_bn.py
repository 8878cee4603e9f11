"""BN-backward pass microbenchmark (HBM-bound): reduce and apply at U-Net sizes.
    python tools/bench_bn.py [--batch 32]
Prints ms and achieved GB/s (algorithmic bytes: reduce 4 B, apply 6 B per bf16 element)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnn_itmo_amd import ops  # noqa: E402

SIZES = [("dec9", 1088, 1920, 64), ("enc1b", 1088, 1920, 32), ("dec8", 544, 960, 128), ("dec7", 272, 480, 256),
         ("dec6", 136, 240, 512)]


def timeit(fn, iters=5):
    fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    dt, T = ops.DTYPES["bfloat16"]
    for name, h, w, c in SIZES:
        n = a.batch
        P = n * h * w
        dy = ops.new_view(n, h, w, c, T)
        dy.buf.uniform_(-1, 1)
        r = torch.rand(P * c, device="cuda").to(T)
        mean = torch.zeros(c, device="cuda")
        inv = torch.ones(c, device="cuda")
        rows = ops.bn_bwd_rows(P, c)
        part = torch.empty(rows * 2 * c, device="cuda")
        coef = torch.ones(3 * c, device="cuda")
        dz = torch.empty(P * c, dtype=T, device="cuda")
        part2 = torch.empty(rows * c, device="cuda")
        tr = timeit(lambda: ops.bn_bwd_reduce(dt, dy, r, c, mean, inv, 0, 0, 0, part))
        ta = timeit(lambda: ops.bn_bwd_apply(dt, dy, r, c, coef, 0, 0, 0, dz, part2))
        el = P * c
        print(f"{name:6s} reduce {tr:7.2f} ms {4 * el / tr / 1e6:7.0f} GB/s   apply {ta:7.2f} ms {6 * el / ta / 1e6:7.0f} GB/s")
        del dy, r, dz
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
