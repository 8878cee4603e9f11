"""Inference CLI: predict.py's I/O conventions, batched.

/root/reference/predict.py:59 reads PNGs as float64 /255; :62 predicts; :64
writes (pred*255).astype('uint8') (truncation).  CPU tests drive the host side
(PNG decode, batching by size, truncation, naming) with a model stand-in whose
predict() is the numpy oracle; the GPU test runs the real HIP path from a Keras
HDF5 checkpoint and compares the PNGs with the oracle's."""
import contextlib
import io
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import cnn_itmo_amd as C  # noqa: E402
from cnn_itmo_amd import predict as PR  # noqa: E402
from oracle import unet_ref as R  # noqa: E402


def _write_pngs(d, frames):
    from PIL import Image
    os.makedirs(d, exist_ok=True)
    names = []
    for i, f in enumerate(frames):
        p = os.path.join(d, f"{i:04d}.png")
        Image.fromarray(f).save(p)
        names.append(p)
    return names


def test_io_conventions_match_reference():
    u8 = np.arange(256, dtype=np.uint8).reshape(16, 16, 1).repeat(3, 2)
    np.testing.assert_array_equal(PR.to_input(u8), R.png_to_input(u8).astype(np.float32))
    pred = np.array([0.0, 0.5, 0.999, 1.0, 0.0039215], np.float32)
    np.testing.assert_array_equal(PR.to_png(pred), R.output_to_png(pred))
    assert PR.to_png(np.float32([0.9999]))[0] == 254  # truncation: max 254 as in output/*.png


class _OracleModel:
    """Stand-in with the Model surface predict_dir uses; predict = fp64 oracle."""

    def __init__(self, m):
        self.inputs = m.inputs
        self.dtype = "float32"
        self.P = m.named_weights()
        self.calls = []

    def predict(self, x, batch_size=32):
        self.calls.append(x.shape)
        H = self.inputs[0].shape[0]
        xp = np.zeros((x.shape[0], H) + x.shape[2:])
        xp[:, :x.shape[1]] = x  # the engine zero-pads short frames (engine.py _input)
        y = R.UNetRef(self.P).forward(xp, training=False)[:, :x.shape[1]]
        return y.astype(np.float32)


def test_predict_dir_host_logic(tmp_path):
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(32, 32, 3), seed=3, verbose=False)
    om = _OracleModel(m)
    rng = np.random.default_rng(0)
    frames = [rng.integers(0, 256, (32, 32, 3), dtype=np.uint8) for _ in range(3)]
    frames += [rng.integers(0, 256, (24, 32, 3), dtype=np.uint8)]  # 8 rows short: engine-padded
    _write_pngs(str(tmp_path / "in"), frames)
    out = PR.predict_dir(om, str(tmp_path / "in"), str(tmp_path / "out"), batch=2, log=lambda *a: None)
    assert [os.path.basename(p) for p in out] == ["0000.png", "0001.png", "0002.png", "0003.png"]
    assert om.calls == [(2, 32, 32, 3), (1, 32, 32, 3), (1, 24, 32, 3)]
    from PIL import Image
    for p, f in zip(out, frames):
        got = np.asarray(Image.open(p))
        if f.shape[0] == 32:
            ref = R.output_to_png(R.UNetRef(om.P).forward(R.png_to_input(f)[None], training=False)[0])
            np.testing.assert_array_equal(got, ref)
        assert got.shape == f.shape and got.dtype == np.uint8


def test_model_for_size_rebuilds_with_shared_weights():
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(32, 32, 3), seed=3, verbose=False)
    assert PR.model_for_size(m, 32, 32) is m and PR.model_for_size(m, 20, 32) is m
    m2 = PR.model_for_size(m, 40, 50)
    assert m2.inputs[0].shape == (48, 64, 3)
    a, b = m.named_weights(), m2.named_weights()
    assert all(np.array_equal(a[k], b[k]) for k in a)


@pytest.mark.gpu
def test_predict_cli_end_to_end_gpu(tmp_path):
    """Keras HDF5 checkpoint -> CLI -> PNGs == oracle PNGs (<= 1 LSB where the fp32
    product sits on a truncation boundary)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(64, 64, 3), seed=5, verbose=False)
    rng = np.random.default_rng(2)
    upd = {k: rng.uniform(0.5, 1.5, v.shape) for k, v in m.named_weights().items() if k.endswith("/moving_variance")}
    m.set_named_weights(upd)
    ck = str(tmp_path / "saved7-model-218-0.73.hdf5")
    m.save(ck)
    frames = [rng.integers(0, 256, (64, 64, 3), dtype=np.uint8) for _ in range(3)]
    frames.append(rng.integers(0, 256, (40, 72, 3), dtype=np.uint8))  # rebuilt for 48x80
    _write_pngs(str(tmp_path / "in"), frames)
    assert PR.main(["--model", ck, "--input", str(tmp_path / "in"), "--output", str(tmp_path / "out"),
                    "--batch", "2"]) == 0
    from PIL import Image
    P = m.named_weights()
    for i, f in enumerate(frames):
        got = np.asarray(Image.open(str(tmp_path / "out" / f"{i:04d}.png"))).astype(int)
        h, w = f.shape[:2]
        x = np.zeros((1, -(-h // 16) * 16, -(-w // 16) * 16, 3))
        x[0, :h, :w] = R.png_to_input(f)
        ref = R.output_to_png(R.UNetRef(P).forward(x, training=False)[0, :h, :w]).astype(int)
        d = np.abs(got - ref)
        assert d.max() <= 1 and (d > 0).mean() < 5e-3, (i, d.max(), (d > 0).mean())
