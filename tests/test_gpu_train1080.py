"""The training composition at the benchmarked frame size against the oracle: ONE fp32
training step (main.py:126-132 trains Keras in fp32) of U_net(input_size=(1080, 1920, 3),
pad=True, dtype="float32") -- the real engine's planner, fused launches, coefficient
buffers, split skip gradients and deferred pool routes at 1088 x 1920 -- on the reference's
12 SDR frames tiled into one real-content frame, against the fp64 oracle of the same step
(tests/golden/train1080.npz, made by tests/golden/make_train1080.py from
tools/train1080_oracle.py; the 89 MB of fp64 gradients are kept as norms plus 4096 fixed
samples per large tensor, every value of the small ones).

Bounds, as the 128x128 test's (test_gpu_model.py::test_unet_train_step_all_74_grads_128):
each of the 74 gradients within rel-L2 max(1e-4, 3x numpy-fp32's own deviation from fp64)
(estimated from the samples for tensors above 4096 entries, with 25 % slack for the
estimate; its L2 norm within the same bound exactly); the loss within max(1e-5, 3x numpy-
fp32's) relative; the Keras moving statistics after the step within rel-L2 max(1e-6, 3x
numpy-fp32's).  At 1080p one frame's BN statistics are still ill-conditioned in the deep
layers (numpy-fp32 deviates up to 0.5 from fp64 on the bottleneck's weight gradients; the
biases before a BN have a zero exact gradient, pure rounding), so the fp32 floor, not a
fixed number, sets the bound, exactly as at 128x128."""
import contextlib
import io
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def _rel(a, b):
    return float(np.linalg.norm(a - b)) / max(float(np.linalg.norm(b)), 1e-300)


@pytest.mark.timeout(600)
def test_train1080_fp32_step_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cnn_itmo_amd as C
    from train1080_oracle import H, SEED, W, inputs
    z = np.load(os.path.join(ROOT, "tests", "golden", "train1080.npz"), allow_pickle=False)
    P, x, t = inputs()
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(H, W, 3), pad=True, dtype="float32", verbose=False)
    m.set_named_weights(P)
    eng = m._engine()
    la = eng.train_step(torch.tensor(x, dtype=torch.float32).cuda(), torch.tensor(t, dtype=torch.float32).cuda(),
                        seed=SEED, apply=False).cpu().numpy().astype(np.float64)
    grads = eng.get_grads()
    after = m.named_weights()
    C.clear_session()

    l64, l32 = float(z["loss64"]), float(z["loss32"])
    lbound = max(1e-5, 3 * abs(l32 - l64) / l64)
    print(f"loss gpu {la[0]:.9f} oracle {l64:.9f} (numpy fp32 {l32:.9f}): rel {abs(la[0] - l64) / l64:.2e} "
          f"<= {lbound:.2e};  acc gpu {la[1]:.6f} oracle {float(z['acc64']):.6f}")
    assert abs(la[0] - l64) <= lbound * l64

    bad = {}
    names = sorted(k[6:] for k in z.files if k.startswith("val/g/"))
    assert len(names) == 74 and set(names) == set(grads)
    for k in names:
        g = grads[k].reshape(-1).astype(np.float64)
        nref, floor = float(z["norm/g/" + k]), float(z["floor/g/" + k])
        bound = max(1e-4, 3 * floor)
        v = z["val/g/" + k]
        if ("idx/g/" + k) in z.files:  # sampled: ||e||^2 ~ N/S * sum over the samples
            idx = z["idx/g/" + k]
            err = float(np.sqrt(g.size / idx.size * np.sum((g[idx] - v) ** 2))) / max(nref, 1e-300)
            ok = err <= 1.25 * bound
        else:
            err = _rel(g, v)
            ok = err <= bound
        nerr = abs(float(np.linalg.norm(g)) - nref) / max(nref, 1e-300)
        ok = ok and nerr <= bound
        print(f"{k:40s} rel-L2 {err:.2e}  |norm| {nerr:.2e}  floor {floor:.2e}  ratio {err / max(floor, 1e-12):.2f}")
        if not ok:
            bad[k] = (err, nerr, floor)
    for k in sorted(n[6:] for n in z.files if n.startswith("val/m/")):
        floor = float(z["floor/m/" + k])
        err = _rel(np.asarray(after[k], np.float64).reshape(-1), z["val/m/" + k])
        print(f"{k:40s} rel-L2 {err:.2e}  floor {floor:.2e}")
        if err > max(1e-6, 3 * floor):
            bad[k] = (err, floor)
    assert not bad, bad
