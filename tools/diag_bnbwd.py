"""Diagnostic: capture bn_bwd inputs/outputs of the first backward block and
recompute dz with the oracle formula from the GPU's own dy and r."""
import io, contextlib, sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import unet_ref as R
import cnn_itmo_amd as C
from cnn_itmo_amd import ops

cap = []
orig_apply = ops.bn_bwd_apply
orig_fin = ops.bn_bwd_finalize
def fin(part, rows, c, count, gamma, mean, inv, dgamma, dbeta, coef):
    orig_fin(part, rows, c, count, gamma, mean, inv, dgamma, dbeta, coef)
    cap.append(dict(part=part.clone(), rows=rows, coef=coef.clone(), mean=mean.clone(), inv=inv.clone(), gamma=gamma.clone(), count=count))
def app(dt, dy, r, c, coef, flags, seed, layer, dz, part):
    orig_apply(dt, dy, r, c, coef, flags, seed, layer, dz, part)
    cap[-1].update(dy=dy.tensor().clone(), r=r.clone(), dz=dz.clone(), c=c)
ops.bn_bwd_apply = app
ops.bn_bwd_finalize = fin
import cnn_itmo_amd.engine as E
E.ops = ops

rng = np.random.default_rng(2)
C.clear_session()
with contextlib.redirect_stdout(io.StringIO()):
    m = C.U_net(input_size=(64, 64, 3), dtype="float32", seed=3)
x = rng.integers(0, 256, size=(2, 64, 64, 3)) / 255.0
t = rng.uniform(size=x.shape)
eng = m._engine()
eng.train_step(torch.tensor(x, dtype=torch.float32).cuda(), torch.tensor(t, dtype=torch.float32).cuda(), seed=77, apply=False)
torch.cuda.synchronize()
for i, d in enumerate(cap[:3]):
    c = d["c"]
    dy = d["dy"].double().cpu().numpy().reshape(-1, c)
    r = d["r"].double().cpu().numpy().reshape(-1, c)
    dz = d["dz"].double().cpu().numpy().reshape(-1, c)
    mu, var = r.mean(0), r.var(0)
    gam = d["gamma"].double().cpu().numpy()
    dr, dg, db = R.bn_train_bwd(dy, r, gam, mu, var)
    dzr = dr * (r > 0)
    coef = d["coef"].double().cpu().numpy().reshape(3, c)
    part = d["part"].double().cpu().numpy().reshape(d["rows"], 2, c).sum(0)
    print(f"block {i}: C={c} max|dz_ref|={np.abs(dzr).max():.3e} err={np.abs(dz-dzr).max():.3e}")
    print("  sdy gpu/ref", part[0][:4], dy.sum(0)[:4])
    inv = 1/np.sqrt(var + 1e-3)
    print("  sdyr gpu/ref", part[1][:4], (dy * (r - mu) * inv).sum(0)[:4])
    print("  mean gpu/ref", d["mean"].cpu().numpy()[:4], mu[:4], " inv", d["inv"].cpu().numpy()[:4], inv[:4])
    M = r.shape[0]
    a = gam * inv; b = a * inv * part[1] / M; e = b * mu - a * part[0] / M
    print("  coef a", coef[0][:3], a[:3]); print("  coef b", coef[1][:3], b[:3]); print("  coef e", coef[2][:3], e[:3])
    print("  count", d["count"], M)
