"""Keras HDF5 model files: cnn_itmo_amd/hdf5.py + keras_h5.py.

The reference checkpoints with ModelCheckpoint(...hdf5) (main.py:124) and
reloads with keras.models.load_model (predict.py:24).  The independent checker
is the real HDF5 C library (tests/h5lib.py over libhdf5 1.10): it wrote the
committed fixture keras_tinynet.hdf5 (tests/golden/make_hdf5.py), writes more
variants here (chunked + deflate + shuffle, variable-length strings,
libver='latest') for our reader, and reads back every file our writer makes.
CPU only (no kernels run)."""
import json
import os

import numpy as np
import pytest

import cnn_itmo_amd as C
from cnn_itmo_amd import hdf5, keras_h5

import h5lib

GOLD = os.path.join(os.path.dirname(__file__), "golden")
needs_lib = pytest.mark.skipif(h5lib.load() is None, reason="libhdf5 not available")


def _same_weights(a, b):
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_golden_keras_file_loads():
    """A file written by libhdf5 in Keras 2.2.4's layout: config, weights, optimizer."""
    C.clear_session()
    m = C.load_model(os.path.join(GOLD, "keras_tinynet.hdf5"))
    exp = np.load(os.path.join(GOLD, "keras_tinynet_expected.npz"))
    ws = m.get_weights()
    assert len(ws) == 6
    for i, w in enumerate(ws):
        np.testing.assert_array_equal(w, exp[f"w{i}"])
    assert [l.type_name for l in m.layers] == ["InputLayer", "Conv2D", "Conv2D", "Conv2D"]
    assert m.layers[1].kernel_initializer == "he_normal" and m.layers[3].activation == "sigmoid"
    assert m.optimizer is not None and m.optimizer.rho == 0.9 and m.optimizer.epsilon == 1e-7
    acc = m.named_accumulators()
    keys = [f"{l.name}/{w}" for l in m.layers for w, _, tr in l.weight_shapes() if tr]
    from cnn_itmo_amd.model import _to_keras
    for i, k in enumerate(keys):
        l = next(l for l in m.layers if l.name == k.split("/")[0])
        np.testing.assert_array_equal(_to_keras(l, k.split("/")[1], acc[k]), exp[f"a{i}"])


def test_golden_file_structure():
    f = hdf5.File(os.path.join(GOLD, "keras_tinynet.hdf5"))
    assert sorted(f.keys()) == ["model_weights", "optimizer_weights"]
    assert bytes(f.attrs["keras_version"]) == b"2.2.4"
    names = [bytes(x) for x in f["model_weights"].attrs["layer_names"]]
    assert names == [b"input_1", b"conv2d_1", b"conv2d_2", b"conv2d_3"]
    wn = [bytes(x) for x in f["model_weights/conv2d_1"].attrs["weight_names"]]
    assert wn == [b"conv2d_1/kernel:0", b"conv2d_1/bias:0"]
    k = f["model_weights/conv2d_1/conv2d_1/kernel:0"].read()
    assert k.shape == (3, 3, 3, 32) and k.dtype == np.float32
    cfg = json.loads(bytes(f.attrs["model_config"]).decode())
    assert cfg["class_name"] == "Model" and cfg["config"]["output_layers"] == [["conv2d_3", 0, 0]]


@needs_lib
@pytest.mark.parametrize("latest,chunked,vlen", [(False, True, False), (False, False, True),
                                                (False, True, True), (True, False, False),
                                                (True, False, True)])
def test_reader_on_library_variants(tmp_path, latest, chunked, vlen):
    C.clear_session()
    m = C.TinyNet(seed=7)
    p = tmp_path / "m.h5"
    h5lib.write_keras_model(p, m, latest=latest, chunked=chunked, vlen=vlen)
    C.clear_session()
    m2 = C.load_model(str(p))
    _same_weights(m.named_weights(), m2.named_weights())


@needs_lib
def test_unet_writer_read_by_library(tmp_path):
    """Model.save('*.h5') of the full U-Net: libhdf5 reads every weight and the config."""
    C.clear_session()
    u = C.U_net(input_size=(32, 32, 3), verbose=False, seed=5)
    p = tmp_path / "unet.hdf5"
    u.save(str(p))
    lf = h5lib.LibFile(p)
    names = [n.decode() for n in lf.read_str_attr("/model_weights", "layer_names")]
    assert names == [l.name for l in u.layers] and len(names) == 66
    cfg = json.loads(lf.read_str_attr("/", "model_config")[0])
    assert cfg["config"]["name"] == "ReinhardtPrediction"
    kw = dict(zip([f"{l.name}/{w}" for l in u.layers for w, _, _ in l.weight_shapes()], u.get_weights()))
    for l in u.layers:
        for w, _, _ in l.weight_shapes():
            got = lf.read_dataset(f"/model_weights/{l.name}/{l.name}/{w}:0")
            np.testing.assert_array_equal(got, kw[f"{l.name}/{w}"])
    assert lf.read_str_attr("/model_weights/conv2d_1", "weight_names") == [b"conv2d_1/kernel:0",
                                                                           b"conv2d_1/bias:0"]
    lf.close()


def test_unet_roundtrip_and_summary(tmp_path, capsys):
    """Our writer -> our reader: the reference network (model.py:204) survives intact,
    summary() still reproduces layers.txt's counts."""
    C.clear_session()
    u = C.U_net(input_size=(512, 512, 3), verbose=False, seed=2)
    p = tmp_path / "saved7-model-01-0.50.hdf5"
    u.save(str(p))
    C.clear_session()
    u2 = C.load_model(str(p))
    assert u2.name == "ReinhardtPrediction"
    assert [l.name for l in u2.layers] == [l.name for l in u.layers]
    _same_weights(u.named_weights(), u2.named_weights())
    u2.summary()
    out = capsys.readouterr().out
    assert "Total params: 11,166,819" in out and "Non-trainable params: 7,808" in out


def test_save_weights_load_weights_h5(tmp_path):
    C.clear_session()
    a = C.TinyNet(seed=1)
    C.clear_session()
    b = C.TinyNet(seed=2)
    p = tmp_path / "w.h5"
    a.save_weights(str(p))
    b.load_weights(str(p))
    _same_weights(a.named_weights(), b.named_weights())


def test_load_weights_topological_with_shifted_names(tmp_path):
    """Keras 2.2 load_weights(by_name=False) is positional: a model whose layer names
    are shifted (another model was built earlier in the session) still loads; by_name=True
    matches names and skips the file layers the model does not have."""
    C.clear_session()
    a = C.TinyNet(seed=1)  # conv2d_1..3
    p = tmp_path / "w.h5"
    a.save_weights(str(p))
    b = C.TinyNet(seed=2)  # same session: conv2d_4..6
    assert {l.name for l in a.layers}.isdisjoint({l.name for l in b.layers} - {"input_1", "input_2"})
    b.load_weights(str(p))
    for (ka, va), (kb, vb) in zip(sorted(a.named_weights().items()), sorted(b.named_weights().items())):
        assert np.array_equal(va, vb), (ka, kb)
    c = C.TinyNet(seed=3)
    before = {k: v.copy() for k, v in c.named_weights().items()}
    c.load_weights(str(p), by_name=True)  # no layer names in common: nothing changes
    _same_weights(before, c.named_weights())


def test_mismatched_file_raises(tmp_path):
    C.clear_session()
    a = C.TinyNet(seed=1)
    p = tmp_path / "w.h5"
    a.save_weights(str(p))
    C.clear_session()
    u = C.U_net(input_size=(32, 32, 3), verbose=False)
    with pytest.raises(ValueError, match="layers"):
        u.load_weights(str(p))


def test_optimizer_state_roundtrip(tmp_path):
    C.clear_session()
    m = C.TinyNet(seed=4)
    rng = np.random.default_rng(0)
    acc = {k: rng.uniform(size=v.shape).astype(np.float32) for k, v in m.named_weights().items()}
    m._pending_accum = ("named", acc, 5)
    p = tmp_path / "o.hdf5"
    m.save(str(p))
    C.clear_session()
    m2 = C.load_model(str(p))
    got = m2.named_accumulators()
    _same_weights(acc, got)


def test_hdf5_writer_scalar_and_empty(tmp_path):
    w = hdf5.Writer()
    w.attrs["s"] = "x"
    w.attrs["n"] = np.int64(3)
    w.attrs["f"] = 2.5
    g = w.create_group("empty")
    g.attrs["weight_names"] = np.zeros((0,), dtype="S1")
    w.create_dataset("d/e", np.zeros((0, 4), np.float32))
    w.create_dataset("sc", np.float32(1.5))
    p = tmp_path / "x.h5"
    w.save(str(p))
    f = hdf5.File(str(p))
    assert bytes(f.attrs["s"]) == b"x" and int(f.attrs["n"]) == 3 and float(f.attrs["f"]) == 2.5
    assert f["empty"].keys() == [] and f["empty"].attrs["weight_names"].shape == (0,)
    assert f["d/e"].read().shape == (0, 4) and float(f["sc"].read()) == 1.5
    assert hdf5.is_hdf5(str(p)) and not hdf5.is_hdf5(__file__)
