"""Spatially tiled inference on the GPU (cnn_itmo_amd/tiled.py): tiles on a 16-aligned
grid with 96-px halos give the full-frame prediction -- fp32 and bf16, a frame whose
width is padded (600 -> 608), tiling in both dimensions, a partial last tile, and a
window that covers a whole dimension; plus the CLI's --tile path.  The full-frame
path is pinned to the oracle in test_golden.py / test_gpu_model.py."""
import contextlib
import io

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cnn_itmo_amd as C  # noqa: E402
from cnn_itmo_amd import predict as PR  # noqa: E402
from cnn_itmo_amd.tiled import predict_tiled  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(h, w, dtype, seed=4):
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(h, w, 3), pad=True, dtype=dtype, seed=seed, verbose=False)
    rng = np.random.default_rng(seed)
    upd = {}
    for k, v in m.named_weights().items():  # non-trivial inference BN
        if k.endswith("/moving_variance") or k.endswith("/gamma"):
            upd[k] = rng.uniform(0.5, 1.5, v.shape)
        elif k.endswith("/moving_mean") or k.endswith("/beta"):
            upd[k] = rng.normal(0, 0.1, v.shape)
    m.set_named_weights(upd)
    return m


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("shape,tile", [((400, 600), (128, 160)), ((336, 256), (64, 512))])
def test_tiled_equals_full_frame(dtype, shape, tile):
    h, w = shape
    m = _model(h, w, dtype)
    rng = np.random.default_rng(7)
    x = (rng.integers(0, 256, (2, h, w, 3)) / 255).astype(np.float32)
    full = PR.model_for_size(m, h, w).predict(PR._pad_cols(x, -(-w // 16) * 16), batch_size=2)[:, :h, :w]
    tiled = predict_tiled(m, x, tile, batch_size=4)
    assert tiled.shape == (2, h, w, 3)
    d = np.abs(tiled - full)
    # the same kernels compute every pixel's dot products in the same order wherever the
    # pixel sits in its launch: the tiled result is bit-identical
    assert float(d.max()) == 0.0, (dtype, float(d.max()), float((d > 0).mean()))


def test_predict_cli_tiled(tmp_path):
    """--tile gives the same PNGs as the whole-frame CLI."""
    from PIL import Image
    m = _model(272, 304, "float32", seed=6)
    ck = str(tmp_path / "m.hdf5")
    m.save(ck)
    rng = np.random.default_rng(3)
    os_in = tmp_path / "in"
    os_in.mkdir()
    for i in range(2):
        Image.fromarray(rng.integers(0, 256, (270, 300, 3), dtype=np.uint8)).save(str(os_in / f"{i}.png"))
    assert PR.main(["--model", ck, "--input", str(os_in), "--output", str(tmp_path / "a"), "--batch", "2"]) == 0
    assert PR.main(["--model", ck, "--input", str(os_in), "--output", str(tmp_path / "b"), "--batch", "2",
                    "--tile", "32,48"]) == 0  # windows 224 x 240 < 272 x 304
    for i in range(2):
        a = np.asarray(Image.open(str(tmp_path / "a" / f"{i}.png"))).astype(int)
        b = np.asarray(Image.open(str(tmp_path / "b" / f"{i}.png"))).astype(int)
        assert a.shape == b.shape == (270, 300, 3)
        assert np.array_equal(a, b)
