"""examples/main.py -- the reference's training script (main.py) on this
framework -- end to end on a tiny synthetic tree: paired augmenting generators
(GPU warp), fit_generator with validation, CSVLogger, Keras-HDF5
ModelCheckpoint and the end-of-epoch prediction callback; the checkpoint then
reloads through load_model and predicts."""
import contextlib
import io
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pngs(d, n, size, rng):
    from PIL import Image
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        Image.fromarray(rng.integers(0, 256, (size, size, 3), dtype=np.uint8)).save(os.path.join(d, f"{i:03d}.png"))


def test_example_main_runs(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(0)
    S = 32
    for split, n in (("train", 4), ("test", 2)):
        for side in ("input1", "output1"):
            _pngs(str(tmp_path / "data" / split / side / "frames"), n, S, rng)
    _pngs(str(tmp_path / "images_to_predict" / "input"), 2, S, rng)
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import main as M
    cwd = os.getcwd()
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            h = M.main(["--root", str(tmp_path), "--size", str(S), "--steps", "2", "--epochs", "2",
                        "--val-steps", "1", "--dtype", "bfloat16"])
    finally:
        os.chdir(cwd)
    assert len(h.history["loss"]) == 2 and all(np.isfinite(h.history["loss"]))
    assert "val_acc" in h.history
    ck = sorted(p for p in os.listdir(tmp_path) if p.startswith("saved7-model-") and p.endswith(".hdf5"))
    assert len(ck) == 2, ck
    log = (tmp_path / "log.csv").read_text().splitlines()
    assert log[0].startswith("epoch;") and len(log) == 3
    outs = sorted(os.listdir(tmp_path / "images_to_predict" / "output"))
    assert outs == ["epochZZZ0000.png", "epochZZZ0001.png", "epochZZZ1000.png", "epochZZZ1001.png"]
    import cnn_itmo_amd as C
    C.clear_session()
    m = C.load_model(str(tmp_path / ck[-1]))
    y = m.predict(rng.uniform(size=(1, S, S, 3)))
    assert y.shape == (1, S, S, 3) and np.isfinite(y).all()
