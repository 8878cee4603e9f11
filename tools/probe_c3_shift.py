"""Is the first layer's direct forward position-independent?  (GPU)

    python tools/probe_c3_shift.py

Runs cnnitmo_conv_c3_fwd on a frame and on crops of it shifted by whole pixels / rows,
and compares the overlapping interior outputs bit for bit (the border column / row of a
crop sees zero padding instead of the frame's data, so it is excluded).  Prints the max
difference and the fraction of differing values per (dtype, shift).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnn_itmo_amd import _lib as L, ops  # noqa: E402


def run(dt, x, wp, bias, sc, sh, aff):
    n, h, w, _ = x.shape
    T = torch.float32 if dt == L.F32 else torch.bfloat16
    out = ops.new_view(n, h, w, 32, T)
    flags = L.RELU | (L.AFFINE if aff else 0)
    ops.conv_c3_fwd(dt, x.contiguous(), n, h, h, w, wp, bias, out, flags, (sc, sh) if aff else None, None)
    torch.cuda.synchronize()
    return out.buf.view(n, h, w, 32).float().cpu().numpy()


def main():
    rng = np.random.default_rng(0)
    n, h, w = 2, 72, 608
    x = torch.tensor(rng.random((n, h, w, 3), dtype=np.float32)).cuda()
    k = torch.tensor(rng.standard_normal((32, 3, 3, 3)).astype(np.float32) * 0.3).cuda()
    bias = torch.tensor(rng.standard_normal(32).astype(np.float32) * 0.1).cuda()
    sc = torch.tensor(rng.uniform(0.5, 1.5, 32).astype(np.float32)).cuda()
    sh = torch.tensor(rng.normal(0, 0.1, 32).astype(np.float32)).cuda()
    for dt, name in ((L.F32, "f32"), (L.BF16, "bf16")):
        T = torch.float32 if dt == L.F32 else torch.bfloat16
        wp = torch.empty(32 * 32, dtype=T, device="cuda")
        ops.prep_c3(dt, k, 32, wp)
        for aff in (False, True):
            full = run(dt, x, wp, bias, sc, sh, aff)
            for dy, dx in ((0, 16), (0, 256), (0, 4), (4, 0), (1, 0), (8, 48)):
                crop = run(dt, x[:, dy:, dx:], wp, bias, sc, sh, aff)
                a = full[:, dy + 1:h - 1, dx + 1:w - 1]
                b = crop[:, 1:h - dy - 1, 1:w - dx - 1]
                d = np.abs(a - b)
                print(f"{name} aff={int(aff)} shift=({dy},{dx}): max {d.max():.3e}  frac {(d > 0).mean():.4f}")


if __name__ == "__main__":
    main()
