"""Pin the oracle to the committed golden fixtures (CPU), and -- on the GPU --
check the HIP path against the same fixtures (tests/golden/make_golden.py)."""
import contextlib
import io
import os
import sys

import numpy as np
import pytest

from oracle import unet_ref as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
from make_golden import seeded_unet_params  # noqa: E402


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def check_summary(z, prefix, named, rtol=1e-9, atol=1e-12):
    for k in named:
        v = np.asarray(named[k], np.float64).reshape(-1)
        np.testing.assert_allclose(v.sum(), z[f"{prefix}/{k}/sum"], rtol=rtol, atol=atol, err_msg=k)
        np.testing.assert_allclose(v[z[f"{prefix}/{k}/idx"]], z[f"{prefix}/{k}/val"], rtol=rtol, atol=atol, err_msg=k)


def test_oracle_ops_golden():
    z = load("ops.npz")
    np.testing.assert_allclose(R.conv2d_same(z["conv_x"], z["conv_w"], z["conv_b"]), z["conv_y"], atol=1e-12)
    dx, dw, db = R.conv2d_same_bwd(z["conv_x"], z["conv_w"], z["conv_dz"])
    np.testing.assert_allclose(dx, z["conv_dx"], atol=1e-12)
    np.testing.assert_allclose(dw, z["conv_dw"], atol=1e-11)
    np.testing.assert_allclose(R.tconv2x2s2(z["tconv_x"], z["tconv_k"], z["tconv_b"]), z["tconv_y"], atol=1e-12)
    y, idx = R.maxpool2x2(z["pool_x"])
    assert np.array_equal(idx, z["pool_idx"]) and np.array_equal(y, z["pool_y"])
    y, m, v = R.bn_train_fwd(z["bn_r"], z["bn_gamma"], z["bn_beta"])
    np.testing.assert_allclose(y, z["bn_y"], atol=1e-12)
    dr, dg, dbe = R.bn_train_bwd(z["bn_dy"], z["bn_r"], z["bn_gamma"], m, v)
    np.testing.assert_allclose(dr, z["bn_dr"], atol=1e-12)
    assert np.array_equal(R.dropout_keep(7, 1, 4096), z["drop_keep_s7_l1"])
    np.testing.assert_allclose(R.mse_grad_z(z["head_yhat"], z["head_t"]), z["head_dz"], atol=1e-15)
    pn, an = R.rmsprop(z["rms_p"], z["rms_g"], z["rms_a"])
    np.testing.assert_allclose(pn, z["rms_p1"], atol=1e-15)


def test_oracle_tiny_golden():
    z = load("tiny.npz")
    P = {k[2:]: z[k] for k in z.files if k.startswith("w/")}
    net = R.TinyNetRef(P)
    np.testing.assert_allclose(net.forward(z["x"]), z["y"], atol=1e-13)
    loss, acc, g = net.backward(z["t"])
    assert abs(loss - float(z["loss"])) < 1e-14
    for k in g:
        np.testing.assert_allclose(g[k], z["g/" + k], atol=1e-13, err_msg=k)


def test_oracle_unet32_golden():
    z = load("unet32.npz")
    P = seeded_unet_params(*z["w_seed"].tolist())
    check_summary(z, "w", P)
    np.testing.assert_allclose(R.UNetRef(P).forward(z["x"], training=False), z["y_infer"], atol=1e-12)
    net = R.UNetRef(P)
    net.forward(z["x"], training=True, seed=5)
    loss, acc, g = net.backward(z["t"])
    assert abs(loss - float(z["loss"])) < 1e-12
    check_summary(z, "g", g, rtol=1e-7, atol=1e-14)


def test_real_image_fixture_format():
    """predict.py conventions on the reference's own SDR image crop: /255 input,
    (pred*255).astype(uint8) truncation (max 254 < 255 as in the shipped outputs)."""
    z = load("real0010.npz")
    assert z["crop_u8"].dtype == np.uint8 and z["crop_u8"].shape == (128, 128, 3)
    assert np.array_equal(R.output_to_png(z["y"][0].astype(np.float64)), z["y_u8"])
    assert z["y_u8"].max() <= 254


def _png(name):
    from PIL import Image
    with Image.open(os.path.join(GOLD, "sdr512", name)) as im:
        return np.asarray(im.convert("RGB"))


def test_sdr512_fixture_and_oracle():
    """The reference's 12 SDR test frames (predict.py:45-64) at 512x512; the oracle is
    pinned to the fixture's summary on the first frame (all 12 run on the GPU box)."""
    z = load("sdr512.npz")
    names = [str(n) for n in z["names"]]
    assert len(names) == 12
    P = seeded_unet_params(*z["w_seed"].tolist())
    check_summary(z, "w", P)
    for nm in names:
        img = _png(nm)
        assert img.shape == (512, 512, 3) and img.dtype == np.uint8
    nm = names[0]
    y = R.UNetRef(P).forward(R.png_to_input(_png(nm))[None], training=False)
    check_summary(z, "y/" + nm, {"out": y}, rtol=1e-10, atol=1e-13)
    assert np.array_equal(np.bincount(R.output_to_png(y[0]).reshape(-1), minlength=256), z[f"hist/{nm}"])


# ---------------------------------------------------------------------------- GPU
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _unet(size, dtype="float32"):
    import cnn_itmo_amd as C
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        return C.U_net(input_size=size, dtype=dtype, verbose=False)


@pytest.mark.gpu
def test_gpu_tiny_golden():
    torch = _gpu()
    import cnn_itmo_amd as C
    z = load("tiny.npz")
    C.clear_session()
    m = C.TinyNet()
    m.set_named_weights({k[2:]: z[k] for k in z.files if k.startswith("w/")})
    assert float(np.abs(m.predict(z["x"]) - z["y"]).max()) <= 1e-5
    eng = m._engine()
    la = eng.train_step(torch.tensor(z["x"], dtype=torch.float32).cuda(),
                        torch.tensor(z["t"], dtype=torch.float32).cuda(), apply=False).cpu().numpy()
    assert abs(la[0] - float(z["loss"])) <= 1e-5 * float(z["loss"])
    g = eng.get_grads()
    for k in g:
        ref = z["g/" + k]
        assert float(np.abs(g[k].reshape(ref.shape) - ref).max()) <= 1e-4 * float(np.abs(ref).max()), k


@pytest.mark.gpu
def test_gpu_unet32_golden():
    _gpu()
    z = load("unet32.npz")
    P = seeded_unet_params(*z["w_seed"].tolist())
    m = _unet((32, 32, 3))
    m.set_named_weights(P)
    y = m.predict(z["x"])
    assert float(np.abs(y - z["y_infer"]).max()) <= 1e-5
    la = m.train_on_batch(z["x"], z["t"])  # dropout seed = engine step 0
    net_loss = float(z["loss"])
    # the fixture's training loss used dropout seed 5; recompute ours with seed 5 too
    import torch
    m2 = _unet((32, 32, 3))
    m2.set_named_weights(P)
    eng = m2._engine()
    la = eng.train_step(torch.tensor(z["x"], dtype=torch.float32).cuda(),
                        torch.tensor(z["t"], dtype=torch.float32).cuda(), seed=5, apply=False).cpu().numpy()
    assert abs(la[0] - net_loss) <= 1e-5 * net_loss
    g = eng.get_grads()
    for k in g:  # gradient norms: see test_gpu_model.py for the conditioning argument
        v = g[k].reshape(-1).astype(np.float64)
        assert abs(np.linalg.norm(v) - float(z[f"g/{k}/norm"])) <= 2e-2 * float(z[f"g/{k}/norm"]) + 1e-12, k


@pytest.mark.gpu
def test_gpu_real_image_golden():
    """North-star parity on a real SDR input: per-pixel max-abs <= 1e-5 and PSNR
    within 0.01 dB of the CPU reference; uint8 outputs agree except at rounding
    boundaries."""
    _gpu()
    z = load("real0010.npz")
    P = seeded_unet_params(*z["w_seed"].tolist())
    m = _unet((128, 128, 3))
    m.set_named_weights(P)
    x = R.png_to_input(z["crop_u8"])[None]
    y = m.predict(x)
    ref = z["y"].astype(np.float64)
    assert float(np.abs(y - ref).max()) <= 1e-5
    target = x  # PSNR against the input, computed identically for both
    p_gpu = 10 * np.log10(1 / np.mean((y - target) ** 2))
    p_ref = 10 * np.log10(1 / np.mean((ref - target) ** 2))
    assert abs(p_gpu - p_ref) < 0.01
    u8 = R.output_to_png(y[0])
    assert np.mean(u8 != z["y_u8"]) < 1e-3


_SDR = {}


def _sdr512_gpu():
    """GPU fp32 inference of all 12 frames in one batch (predict.py:59-64 conventions)."""
    if not _SDR:
        z = load("sdr512.npz")
        names = [str(n) for n in z["names"]]
        P = seeded_unet_params(*z["w_seed"].tolist())
        m = _unet((512, 512, 3))
        m.set_named_weights(P)
        x = np.stack([R.png_to_input(_png(nm)) for nm in names])
        y = m.predict(x, batch_size=12)
        _SDR.update(z=z, P=P, names=names, y=dict(zip(names, y)))
    return _SDR


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(12))
def test_gpu_sdr512_frames(k):
    """All 12 of the reference's SDR frames at native 512x512 through the fp32 HIP
    path vs the fp64 oracle run here on the same frame: per-pixel max-abs <= 1e-5,
    PSNR(gpu, oracle) >= 100 dB, PSNR against the input within 0.01 dB of the
    oracle's, predict.py:64 uint8 output equal except at truncation boundaries."""
    _gpu()
    s = _sdr512_gpu()
    nm = s["names"][k]
    y = s["y"][nm].astype(np.float64)
    x = R.png_to_input(_png(nm))
    ref = R.UNetRef(s["P"]).forward(x[None], training=False)[0]
    check_summary(s["z"], "y/" + nm, {"out": ref[None]}, rtol=1e-9, atol=1e-12)  # oracle == fixture
    err = float(np.abs(y - ref).max())
    mse = float(np.mean((y - ref) ** 2))
    psnr = 10 * np.log10(1.0 / max(mse, 1e-300))
    p_gpu = 10 * np.log10(1 / np.mean((y - x) ** 2))
    p_ref = 10 * np.log10(1 / np.mean((ref - x) ** 2))
    u8, u8r = R.output_to_png(y), R.output_to_png(ref)
    print(f"{nm}: max-abs {err:.2e}, PSNR(gpu, oracle) {psnr:.1f} dB, |dPSNR| {abs(p_gpu - p_ref):.2e} dB, "
          f"uint8 mismatches {int(np.sum(u8 != u8r))}")
    assert err <= 1e-5
    assert psnr >= 100.0
    assert abs(p_gpu - p_ref) < 0.01
    assert np.mean(u8 != u8r) < 1e-3 and np.abs(u8.astype(int) - u8r).max() <= 1


@pytest.mark.gpu
def test_gpu_sdr1080_mosaic():
    """The north star's parity at the benchmarked frame size, end to end: the 12 SDR
    frames' centre crops tiled into ONE real-content 1080x1920 frame
    (make_golden.mosaic1080) through U_net(input_size=(1080, 1920, 3), pad=True,
    dtype="float32").predict on the GPU, against the fp64 oracle on the host with the
    same zero-pad to 1088 rows and crop (predict.py:59-64, model.py:204-278).  The
    oracle's output is pinned to the committed sdr1080.npz summary first.
    Bounds: per-pixel max-abs <= 1e-5, PSNR(gpu, oracle) >= 100 dB, PSNR against the
    input within 0.01 dB of the oracle's, predict.py:64 uint8 within +-1."""
    _gpu()
    from make_golden import mosaic1080, oracle_padded
    import cnn_itmo_amd as C
    z = load("sdr1080.npz")
    names = [str(n) for n in z["names"]]
    P = seeded_unet_params(*z["w_seed"].tolist())
    x = R.png_to_input(mosaic1080([_png(nm) for nm in names]))[None]
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(1080, 1920, 3), pad=True, dtype="float32", verbose=False)
    m.set_named_weights(P)
    y = m.predict(x).astype(np.float64)
    C.clear_session()
    assert y.shape == (1, 1080, 1920, 3)
    ref = oracle_padded(P, x)
    check_summary(z, "y", {"out": ref}, rtol=1e-9, atol=1e-12)  # oracle == fixture
    err = float(np.abs(y - ref).max())
    psnr = 10 * np.log10(1.0 / max(float(np.mean((y - ref) ** 2)), 1e-300))
    p_gpu = 10 * np.log10(1 / np.mean((y - x) ** 2))
    p_ref = 10 * np.log10(1 / np.mean((ref - x) ** 2))
    assert abs(p_ref - float(z["psnr_vs_input"])) < 1e-9
    u8, u8r = R.output_to_png(y[0]), R.output_to_png(ref[0])
    print(f"1080x1920 mosaic: max-abs {err:.2e}, PSNR(gpu, oracle) {psnr:.1f} dB, |dPSNR| {abs(p_gpu - p_ref):.2e} dB, "
          f"uint8 mismatches {int(np.sum(u8 != u8r))} of {u8.size}")
    assert err <= 1e-5
    assert psnr >= 100.0
    assert abs(p_gpu - p_ref) < 0.01
    assert np.abs(u8.astype(int) - u8r).max() <= 1
