"""Debug: BN partial sums of the first halo conv launch vs the stored output and
vs an exact fp64 conv of the launch's inputs (small frame)."""
import contextlib
import io
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import cnn_itmo_amd as C  # noqa: E402
from cnn_itmo_amd import _lib as L, ops  # noqa: E402

F64 = torch.float64
orig = ops.conv3x3_fwd
done = []


def wrapped(dt, x, wt, bias, out, flags=0, aff=None, stats=None, border=None):
    orig(dt, x, wt, bias, out, flags, aff, stats, border)
    torch.cuda.synchronize()
    if done or stats is None:
        return
    done.append(1)
    n, h, w, cin, cout = x.n, x.h, x.w, x.c, out.c
    xt = x.tensor().to(F64)
    xp = torch.nn.functional.pad(xt, (0, 0, 1, 1, 1, 1))
    W = wt.view(cout, 3, 3, cin).to(F64)
    z = torch.zeros(n, h, w, cout, dtype=F64, device="cuda")
    for r in range(3):
        for s in range(3):
            z += xp[:, r:r + h, s:s + w] @ W[:, r, s].t()
    z += bias.to(F64)
    if border is not None:
        oh = torch.arange(h, device="cuda")[:, None].expand(h, w).reshape(-1)
        ow = torch.arange(w, device="cuda")[None, :].expand(h, w).reshape(-1)
        from launch_check import _border_corr
        z -= _border_corr(border, oh, ow, h, w).view(1, h, w, cout)
    z = z.clamp_min(0)
    o = out.tensor().to(F64)
    tot = stats.view(-1, 2, cout).to(F64).sum(0)
    print("rows", stats.numel() // (2 * cout), "flags", flags, "border", border is not None)
    print("max |stored - exact|", float((o - z).abs().max()), "rel", float((o - z).abs().max() / z.abs().max()))
    print("stats vs exact sum  (rel):", ((tot[0] - z.sum((0, 1, 2))) / z.sum((0, 1, 2))).abs().max().item())
    print("stats vs stored sum (rel):", ((tot[0] - o.sum((0, 1, 2))) / o.sum((0, 1, 2))).abs().max().item())
    print("stored vs exact sum (rel):", ((o.sum((0, 1, 2)) - z.sum((0, 1, 2))) / z.sum((0, 1, 2))).abs().max().item())
    print("stats row sums first rows:", stats.view(-1, 2, cout)[:4, 0, :4])
    d = (tot[0] - z.sum((0, 1, 2)))
    print("per-channel abs diff", d[:8])
    # where does the stored output differ: per row / column sums
    e = (o - z).sum((0, 3))
    print("row error sums", e.sum(1)[:4], e.sum(1)[-4:], "col error sums", e.sum(0)[:4], e.sum(0)[-4:])


ops.conv3x3_fwd = wrapped
C.clear_session()
with contextlib.redirect_stdout(io.StringIO()):
    m = C.U_net(input_size=(72, 112, 3), pad=True, dtype=os.environ.get("DT", "bfloat16"), seed=0, verbose=False)
eng = m._engine()
g = torch.Generator(device="cuda")
g.manual_seed(11)
x = torch.randint(0, 256, (2, 72, 112, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
t = torch.randint(0, 256, (2, 72, 112, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
eng.train_step(x, t, seed=3)
torch.cuda.synchronize()
