"""Noise floor: numpy float32 run of the oracle vs fp64 on the U-Net train-step case
of tests/test_gpu_model.py (justifies the fp32 gradient tolerance)."""
import sys; sys.path.insert(0, ".")
import numpy as np, io, contextlib
from oracle import unet_ref as R
import cnn_itmo_amd as C
rng = np.random.default_rng(2)
C.clear_session()
with contextlib.redirect_stdout(io.StringIO()):
    m = C.U_net(input_size=(64, 64, 3), dtype="float32", seed=3)
P = m.named_weights()
x = rng.integers(0, 256, size=(2, 64, 64, 3)) / 255.0
t = rng.uniform(size=x.shape)
n64 = R.UNetRef(P, np.float64); n64.forward(x, True, seed=77); l64, a64, g64 = n64.backward(t)
n32 = R.UNetRef(P, np.float32); n32.forward(x.astype(np.float32), True, seed=77); l32, a32, g32 = n32.backward(t.astype(np.float32))
rows = []
for k in g64:
    d = np.abs(g32[k] - g64[k]).max() / np.abs(g64[k]).max()
    l2 = np.linalg.norm(g32[k] - g64[k]) / np.linalg.norm(g64[k])
    rows.append((d, l2, k))
for r in sorted(rows, reverse=True)[:12]: print(f"{r[0]:.3e} l2={r[1]:.3e} {r[2]}")
print("loss", l64, l32)
