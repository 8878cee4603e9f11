"""End-to-end parity of the U-Net hot path on the GPU (HIP kernels via the C ABI)
against the numpy oracle in fp64, same seeded weights and inputs.

Tolerances (stated per north star):
  fp32 inference: per-pixel max-abs <= 1e-4 and PSNR(gpu, target) within 0.01 dB
  of PSNR(oracle, target).
  fp32 training: loss rel <= 1e-5; the worst per-tensor gradient rel-L2 must be
  no worse than that of numpy's own float32 run of the same oracle (and <= 2e-2).
  Why self-calibrating: training-mode BN over near-degenerate channels (batch
  variance << eps, e.g. conv2d_9 at 4x4x2 pixels) amplifies fp32 rounding ~30x
  per layer, so fp32 gradients of this net are only ~1e-2 accurate against fp64
  whoever computes them (tools/noise_floor.py); the per-kernel tests
  (test_gpu_ops.py) pin every kernel at 1e-4 in isolation.  After one RMSprop
  step the weights equal RMSprop applied to the GPU's own gradients (atol 1e-6).
  bf16 (bf16 storage, fp32 accumulation): output max-abs <= 3e-2; one step: loss
  rel <= 2e-2 and the head's gradients rel-L2 <= 0.1; functional: bf16 training
  tracks fp32 training (final loss within 10%)."""
import os
import io
import contextlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import unet_ref as R  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def build_unet(size, dtype, seed=1):
    import cnn_itmo_amd as C
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=size, dtype=dtype, seed=seed)
    return m


def randomize_bn(m, rng):
    named = m.named_weights()
    upd = {}
    for k, v in named.items():
        if k.endswith("/moving_mean"):
            upd[k] = rng.uniform(0, 1, v.shape)
        elif k.endswith("/moving_variance"):
            upd[k] = rng.uniform(0.5, 2, v.shape)
        elif k.endswith("/gamma"):
            upd[k] = rng.uniform(0.5, 1.5, v.shape)
        elif k.endswith("/beta"):
            upd[k] = rng.uniform(-0.2, 0.2, v.shape)
        elif k.endswith("/bias"):
            upd[k] = rng.uniform(-0.1, 0.1, v.shape)
    m.set_named_weights(upd)
    return m.named_weights()


def psnr(a, b):
    mse = float(np.mean((a - b) ** 2))
    return 10 * np.log10(1.0 / mse) if mse > 0 else float("inf")


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_unet_inference_parity(dtype):
    rng = np.random.default_rng(0)
    m = build_unet((64, 64, 3), dtype)
    P = randomize_bn(m, rng)
    x = rng.integers(0, 256, size=(2, 64, 64, 3)) / 255.0
    t = rng.uniform(size=x.shape)
    y = m.predict(x)
    ref = R.UNetRef(P).forward(x, training=False)
    err = float(np.abs(y - ref).max())
    if dtype == "float32":
        assert err <= 1e-4, err
        assert abs(psnr(y, t) - psnr(ref, t)) < 0.01
    else:
        assert err <= 3e-2, err


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_fused_head_paths_agree(dtype):
    """The head is computed on every inference path: predict / predict_into (head fused into
    conv9's epilogue, engine.py _plan_head_fusion) and a bare forward + HeadStage.infer (the
    stand-alone head kernel, since no fused head ran in that forward) give the same frames."""
    rng = np.random.default_rng(4)
    m = build_unet((64, 96, 3), dtype)
    P = randomize_bn(m, rng)
    e = m._engine()
    # fp32: conv9 reads the zero-copy [conv1 | up9] concat, so the fused head applies; bf16
    # splits that concat over two sources (conv3x3_fwd_cat), which EPI 3 does not take
    assert e.stages[-1].fused == (dtype == "float32")
    x = torch.tensor(rng.integers(0, 256, size=(2, 64, 96, 3)) / 255.0, dtype=torch.float32).cuda()
    y_fused = torch.full((2, 64, 96, 3), -1.0, device="cuda")
    e.predict_into(x, y_fused)
    assert e.stages[-1].vin.producer.head_ran == e.stages[-1].fused
    y_plain = torch.full((2, 64, 96, 3), -1.0, device="cuda")
    n = e.forward(x, training=False)
    assert not e.stages[-1].vin.producer.head_ran
    e.stages[-1].infer(n, y_plain)
    e._release()
    torch.cuda.synchronize()
    a, b = y_fused.cpu().numpy(), y_plain.cpu().numpy()
    assert a.min() >= 0.0 and b.min() >= 0.0  # every value written (the -1 fill is gone)
    ref = R.UNetRef(P).forward(x.cpu().numpy().astype(np.float64), training=False)
    tol = 1e-4 if dtype == "float32" else 3e-2
    assert float(np.abs(a - ref).max()) <= tol
    assert float(np.abs(b - ref).max()) <= tol
    # the two heads differ only by the summation order of the 64-channel dot product
    # (fp32) or by the bf16 rounding of the stored conv output (bf16)
    assert float(np.abs(a - b).max()) <= (1e-5 if dtype == "float32" else 3e-2)
    with pytest.raises(ValueError):
        e.predict_into(x, torch.empty((2, 64, 96, 4), device="cuda"))


def test_unet_inference_padded_1080_style():
    """H not divisible by 16: pad=True model, zero-padded rows, cropped output."""
    import cnn_itmo_amd as C
    rng = np.random.default_rng(1)
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(56, 48, 3), pad=True, seed=2)
    assert m.input_shape == (None, 64, 48, 3)
    P = randomize_bn(m, rng)
    x = rng.uniform(size=(1, 56, 48, 3))
    y = m.predict(x)
    xp = np.zeros((1, 64, 48, 3))
    xp[:, :56] = x
    ref = R.UNetRef(P).forward(xp, training=False)[:, :56]
    assert y.shape == (1, 56, 48, 3)
    assert float(np.abs(y - ref).max()) <= 1e-4


def _grad_err(g, r):
    return float(np.abs(g - r).max()) / max(1e-12, float(np.abs(r).max()))


def _rel_l2(g, r):
    return float(np.linalg.norm(g - r)) / max(1e-12, float(np.linalg.norm(r)))


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_unet_train_step_parity(dtype):
    rng = np.random.default_rng(2)
    m = build_unet((64, 64, 3), dtype, seed=3)
    P = randomize_bn(m, rng)
    x = rng.integers(0, 256, size=(2, 64, 64, 3)) / 255.0
    t = rng.uniform(size=x.shape)
    eng = m._engine()
    seed = 77
    la = eng.train_step(torch.tensor(x, dtype=torch.float32).cuda(),
                        torch.tensor(t, dtype=torch.float32).cuda(), seed=seed).cpu().numpy()
    grads = eng.get_grads()
    after = m.named_weights()
    net = R.UNetRef(P)
    net.forward(x, training=True, seed=seed)
    loss, acc, rg = net.backward(t)
    net.apply_rmsprop(rg, {})
    assert set(rg) == set(grads)
    if dtype == "float32":
        assert abs(la[0] - loss) <= 1e-5 * loss
        assert abs(la[1] - acc) <= 1.0 / x[..., 0].size + 1e-7
        n32 = R.UNetRef(P, np.float32)
        n32.forward(x.astype(np.float32), training=True, seed=seed)
        _, _, g32 = n32.backward(t.astype(np.float32))
        floor = max(_rel_l2(g32[k], rg[k]) for k in rg)
        worst = max((_rel_l2(grads[k].reshape(rg[k].shape), rg[k]), k) for k in rg)
        print(f"fp32 grad rel-L2: gpu worst {worst}, numpy-fp32 floor {floor:.3e}")
        assert worst[0] <= min(2e-2, max(floor, 1e-3)), (worst, floor)
        # optimizer wiring: weights after the step == RMSprop of the GPU's own gradients
        for k in rg:
            exp, _ = R.rmsprop(P[k].astype(np.float64), grads[k].reshape(P[k].shape).astype(np.float64),
                               np.zeros(P[k].shape))
            np.testing.assert_allclose(after[k], exp, atol=1e-6, err_msg=k)
        for k in after:
            if "moving" in k:
                np.testing.assert_allclose(after[k], net.P[k], atol=1e-5, rtol=1e-5, err_msg=k)
    else:
        assert abs(la[0] - loss) <= 2e-2 * loss
        for k in ("conv2d_15/kernel", "conv2d_15/bias", "batch_normalization_18/gamma",
                  "batch_normalization_18/beta"):
            assert _rel_l2(grads[k].reshape(rg[k].shape), rg[k]) <= 0.1, k


def test_bf16_training_tracks_fp32():
    """The bench dtype: 12 bf16 steps follow the fp32 loss trajectory."""
    rng = np.random.default_rng(11)
    x = rng.integers(0, 256, size=(4, 32, 32, 3)) / 255.0
    t = np.clip(x ** 2.2 * 1.3, 0, 1)
    curves = {}
    for dtype in ("float32", "bfloat16"):
        m = build_unet((32, 32, 3), dtype, seed=12)
        eng = m._engine()
        xs, ts = torch.tensor(x, dtype=torch.float32).cuda(), torch.tensor(t, dtype=torch.float32).cuda()
        curves[dtype] = [eng.train_step(xs, ts, seed=i)[0].item() for i in range(12)]
    f, b = curves["float32"], curves["bfloat16"]
    assert f[-1] < f[0] and b[-1] < b[0], curves
    assert abs(b[-1] - f[-1]) <= 0.1 * f[-1], curves


def test_unet_two_steps_and_determinism():
    """Two fp32 steps track the oracle; the same seeds give bitwise-equal results."""
    rng = np.random.default_rng(4)
    x = rng.uniform(size=(2, 32, 32, 3))
    t = rng.uniform(size=x.shape)
    outs = []
    for _ in range(2):
        m = build_unet((32, 32, 3), "float32", seed=5)
        eng = m._engine()
        xs, ts = torch.tensor(x, dtype=torch.float32).cuda(), torch.tensor(t, dtype=torch.float32).cuda()
        l1 = eng.train_step(xs, ts, seed=1).cpu().numpy()
        l2 = eng.train_step(xs, ts, seed=2).cpu().numpy()
        outs.append((l1, l2, eng.params.cpu().numpy()))
    assert np.array_equal(outs[0][2], outs[1][2])
    P = build_unet((32, 32, 3), "float32", seed=5).named_weights()
    ref = {}
    for dt in (np.float64, np.float32):
        net = R.UNetRef(P, dt)
        acc = {}
        ref[dt] = (net.train_step(x.astype(dt), t.astype(dt), acc, seed=1)[0],
                   net.train_step(x.astype(dt), t.astype(dt), acc, seed=2)[0])
    r1, r2 = ref[np.float64]
    assert abs(outs[0][0][0] - r1) <= 1e-5 * r1
    # the first RMSprop step is sign-like (|update| ~ lr/sqrt(1-rho) for every weight), so the
    # second loss inherits the sign noise of near-zero gradients: calibrate on numpy-fp32's own
    # deviation from fp64 (1.4e-3 relative on this case).
    floor = abs(ref[np.float32][1] - r2)
    assert abs(outs[0][1][0] - r2) <= max(1e-3 * r2, 3 * floor), (outs[0][1][0], r2, ref[np.float32][1])


def test_tiny_net_config1_parity():
    """BASELINE configs[0]: 64x64, 3-conv net, batch 1 (fp32)."""
    import cnn_itmo_amd as C
    rng = np.random.default_rng(6)
    C.clear_session()
    m = C.TinyNet()
    P = m.named_weights()
    x = rng.uniform(size=(1, 64, 64, 3))
    t = rng.uniform(size=x.shape)
    y = m.predict(x)
    ref = R.TinyNetRef(P)
    assert float(np.abs(y - ref.forward(x)).max()) <= 1e-5
    loss, acc, rg = ref.backward(t)
    eng = m._engine()
    la = eng.train_step(torch.tensor(x, dtype=torch.float32).cuda(), torch.tensor(t, dtype=torch.float32).cuda())
    g = eng.get_grads()
    assert abs(la[0].item() - loss) <= 1e-5 * loss
    for k in rg:  # no BatchNorm here: well conditioned, tight tolerance
        assert _grad_err(g[k].reshape(rg[k].shape), rg[k]) <= 1e-4, k


def test_save_load_roundtrip(tmp_path):
    import cnn_itmo_amd as C
    rng = np.random.default_rng(7)
    m = build_unet((32, 32, 3), "float32", seed=8)
    x = rng.uniform(size=(1, 32, 32, 3))
    m.train_on_batch(x, rng.uniform(size=x.shape))
    y0 = m.predict(x)
    p = str(tmp_path / "m.npz")
    m.save(p)
    m2 = C.load_model(p)
    np.testing.assert_array_equal(m2.predict(x), y0)
    assert m2.count_params() == m.count_params()


@pytest.mark.parametrize("ext", ["npz", "hdf5"])
def test_checkpoint_resume_is_exact(tmp_path, ext):
    """ModelCheckpoint -> load_model -> continue training == uninterrupted training
    (weights, BN moving stats and RMSprop accumulators all round-trip)."""
    import cnn_itmo_amd as C
    rng = np.random.default_rng(3)
    x = rng.uniform(size=(2, 32, 32, 3))
    t = rng.uniform(size=x.shape)
    m = build_unet((32, 32, 3), "float32", seed=4)
    m.train_on_batch(x, t)
    p = str(tmp_path / f"saved7-model-01-0.50.{ext}")
    m.save(p)
    m.train_on_batch(x, t)
    C.clear_session()
    m2 = C.load_model(p)
    m2._engine().step = m._engine().step - 1  # dropout seed follows the step counter
    m2.train_on_batch(x, t)
    a, b = m.named_weights(), m2.named_weights()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_fit_generator_loss_decreases():
    """main.py:126-132 shape of use: fit_generator over a paired generator."""
    rng = np.random.default_rng(9)
    m = build_unet((32, 32, 3), "float32", seed=10)
    x = rng.uniform(size=(4, 32, 32, 3))
    t = np.clip(x * 0.8 + 0.1, 0, 1)

    def gen():
        while True:
            yield x[:2], t[:2]
            yield x[2:], t[2:]
    h = m.fit_generator(gen(), steps_per_epoch=10, epochs=3, verbose=0)
    assert h.history["loss"][-1] < h.history["loss"][0]


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_unet_train_step_all_74_grads_128(dtype):
    """Every one of the 74 gradients of one training step at 128x128 b2 (the
    bottleneck sees 8x8x2 pixels per channel), each against the fp64 oracle and
    held to the noise floor of an implementation of that precision:
      fp32: rel-L2 <= max(1e-4, 3x the deviation of numpy's own float32 run of the
      same oracle);  loss rel <= 1e-6.  Measured (round 2): the GPU's fp32 gradients
      are 2e-3..9e-3 from fp64 while numpy-fp32 is 3e-2..9e-2 away -- the chain of 18
      training-mode BN backwards (dy - mean(dy) - rhat*mean(dy*rhat): near-total
      cancellation) amplifies fp32 rounding even at 128x128, so 1e-4 per gradient
      is below what fp32 arithmetic can deliver on this net; the GPU sits 10x under
      the fp32 floor.
      bf16 (the bench dtype): rel-L2 <= max(3x, 2e-3) the deviation of the oracle run
      with bf16 STORAGE emulated (R.round_bf16 at every stored weight, activation and
      gradient, fp64 arithmetic);  loss rel <= 5e-3."""
    rng = np.random.default_rng(21)
    m = build_unet((128, 128, 3), dtype, seed=7)
    P = randomize_bn(m, rng)
    x = rng.integers(0, 256, size=(2, 128, 128, 3)) / 255.0
    t = np.clip(x ** 2.2 * 1.2, 0, 1)
    eng = m._engine()
    seed = 9
    la = eng.train_step(torch.tensor(x, dtype=torch.float32).cuda(),
                        torch.tensor(t, dtype=torch.float32).cuda(), seed=seed, apply=False).cpu().numpy()
    grads = eng.get_grads()
    net = R.UNetRef(P)
    net.forward(x, training=True, seed=seed)
    loss, acc, rg = net.backward(t)
    assert len(rg) == 74 and set(rg) == set(grads)
    err = {k: _rel_l2(grads[k].reshape(rg[k].shape), rg[k]) for k in rg}
    if dtype == "float32":
        em = R.UNetRef(P, np.float32)
        em.forward(x.astype(np.float32), training=True, seed=seed)
        eloss, _, eg = em.backward(t.astype(np.float32))
    else:
        em = R.UNetRef(P, store=R.round_bf16)
        em.forward(x, training=True, seed=seed)
        eloss, _, eg = em.backward(t)
    floor = {k: _rel_l2(eg[k], rg[k]) for k in rg}
    for k in sorted(rg):
        print(f"{dtype} {k:40s} gpu {err[k]:.2e}  floor {floor[k]:.2e}  ratio {err[k] / max(floor[k], 1e-12):.2f}")
    print(f"{dtype} loss rel {abs(la[0] - loss) / loss:.2e} (floor {abs(eloss - loss) / loss:.2e})")
    if dtype == "float32":
        assert abs(la[0] - loss) <= 1e-6 * loss
        bad = {k: (err[k], floor[k]) for k in rg if err[k] > max(1e-4, 3 * floor[k])}
        tight = sum(err[k] <= 1e-4 for k in rg)
        print(f"fp32: {tight}/74 gradients within rel-L2 1e-4")
    else:
        assert abs(la[0] - loss) <= 5e-3 * loss
        bad = {k: (err[k], floor[k]) for k in rg if err[k] > max(3 * floor[k], 2e-3)}
    assert not bad, bad


_HALO_OFF = r"""
import contextlib, io, sys, numpy as np, torch
sys.path.insert(0, {root!r})
import cnn_itmo_amd as C
from cnn_itmo_amd.engine import ConcatStage
with contextlib.redirect_stdout(io.StringIO()):
    m = C.U_net(input_size=(64, 64, 3), dtype="bfloat16", seed=3, verbose=False)
rng = np.random.default_rng(0)
x = rng.uniform(size=(2, 64, 64, 3)); t = rng.uniform(size=(2, 64, 64, 3))
la = m.train_on_batch(x, t)
y = m.predict(x)
split = [st.vout.split for st in m._engine().stages if isinstance(st, ConcatStage)]
print("split", split, "loss", la[0], "finite", bool(np.isfinite(y).all()))
"""


@pytest.mark.parametrize("halo", ["1", "0"])
def test_bf16_training_without_halo_kernel(halo):
    """The split level-0 concat (Engine._plan_split_concats) is planned only where its
    two-source forward runs: with the halo kernel disabled (CNNITMO_HALO=0, read once per
    process) the concat stays one buffer and bf16 training and predict still work."""
    import subprocess
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CNNITMO_HALO=halo)
    r = subprocess.run([_sys.executable, "-c", _HALO_OFF.format(root=root)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("split")][-1]
    print(f"CNNITMO_HALO={halo}: {line}")
    assert "finite True" in line
    if halo == "0":
        assert "True" not in line.split("loss")[0], line
