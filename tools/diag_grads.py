"""Diagnostic: per-gradient error of one U-Net train step vs the oracle."""
import io, contextlib, sys
import numpy as np
import torch
sys.path.insert(0, ".")
from oracle import unet_ref as R
import cnn_itmo_amd as C

size = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dtype = sys.argv[2] if len(sys.argv) > 2 else "float32"
rng = np.random.default_rng(2)
C.clear_session()
with contextlib.redirect_stdout(io.StringIO()):
    m = C.U_net(input_size=(size, size, 3), dtype=dtype, seed=3)
P = m.named_weights()
x = rng.integers(0, 256, size=(2, size, size, 3)) / 255.0
t = rng.uniform(size=x.shape)
eng = m._engine()
la = eng.train_step(torch.tensor(x, dtype=torch.float32).cuda(), torch.tensor(t, dtype=torch.float32).cuda(), seed=77, apply=False).cpu().numpy()
g = eng.get_grads()
net = R.UNetRef(P)
net.forward(x, training=True, seed=77)
loss, acc, rg = net.backward(t)
print("loss", la, loss, acc)
rows = []
for k in rg:
    a = g[k].reshape(rg[k].shape); b = rg[k]
    rows.append((float(np.linalg.norm(a - b)) / max(1e-30, float(np.linalg.norm(b))),
                 float(np.abs(a - b).max()) / max(1e-12, float(np.abs(b).max())), k, float(np.abs(b).max())))
order = {k: i for i, k in enumerate(eng.pslices)}
for r in sorted(rows, key=lambda r: order[r[2]]):
    print(f"l2={r[0]:.3e} maxrel={r[1]:.3e}  {r[2]:40s} max|ref|={r[3]:.3e}")
