"""Training-data pipeline: cnn_itmo_amd/datagen.py vs the
keras_preprocessing restatement in oracle/augment_ref.py (random stream) and
scipy.ndimage.affine_transform (the warp Keras calls), main.py:71-98's settings.

CPU: the per-batch index/transform stream, the affine matrices, directory
listing and pairing (the GPU transform is stubbed out).  GPU: the HIP warp
against scipy at max-abs <= 2e-6 (values in [0, 1] after rescale; float64
coordinates on both sides, FMA contraction aside), and zip-paired generators."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from cnn_itmo_amd import datagen as D  # noqa: E402
from oracle import augment_ref as A  # noqa: E402

REF_ARGS = dict(rescale=1. / 255, rotation_range=90, horizontal_flip=True, vertical_flip=True, zoom_range=0.2)
KW = dict(rotation_range=90, zoom_range=(0.8, 1.2), horizontal_flip=True, vertical_flip=True)


class _Capture:
    """Stands in for the GPU transform: records (frames, params)."""

    def __init__(self, gen):
        self.seen = []
        gen.transform_batch = self

    def __call__(self, frames, params, out=None):
        self.seen.append((np.asarray(frames).copy(), params))
        return np.zeros(np.asarray(frames).shape, np.float32)


def test_random_stream_matches_keras_restatement():
    rng = np.random.default_rng(0)
    frames = rng.integers(0, 256, (7, 8, 8, 3), dtype=np.uint8)
    g = D.ImageDataGenerator(**REF_ARGS)
    cap = _Capture(g)
    it = g.flow(frames, batch_size=2, shuffle=True, seed=1)
    nb = 9  # crosses two epoch boundaries (7 frames, batches of 2: 4 per epoch)
    for _ in range(nb):
        next(it)
    saved = np.random.get_state()
    ref = list(A.flow(frames, 2, 1, nb, **KW))
    np.random.set_state(saved)
    assert len(cap.seen) == nb
    for (fr, params), (idx, rparams) in zip(cap.seen, ref):
        np.testing.assert_array_equal(fr, frames[idx])
        for p, q in zip(params, rparams):
            for k in ("theta", "zx", "zy", "flip_horizontal", "flip_vertical"):
                assert p[k] == q[k], k


def test_global_numpy_state_untouched():
    g = D.ImageDataGenerator(**REF_ARGS)
    _Capture(g)
    np.random.seed(123)
    a = np.random.random_sample()
    np.random.seed(123)
    it = g.flow(np.zeros((4, 8, 8, 3), np.uint8), batch_size=2, seed=1)
    next(it)
    assert np.random.random_sample() == a


def test_affine_matches_keras_matrix():
    p = dict(theta=33.0, zx=0.9, zy=1.15, flip_horizontal=1, flip_vertical=0)
    m, fl = D.ImageDataGenerator.affine(p, 40, 24)
    t = np.deg2rad(33.0)
    rot = np.array([[np.cos(t), -np.sin(t), 0], [np.sin(t), np.cos(t), 0], [0, 0, 1]])
    ref = A.transform_matrix_offset_center(rot @ np.diag([0.9, 1.15, 1.0]), 40, 24)
    np.testing.assert_array_equal(m, ref[:2].reshape(-1))
    assert fl == 1
    m, fl = D.ImageDataGenerator.affine(dict(theta=0, zx=1, zy=1, flip_vertical=1), 5, 5)
    np.testing.assert_array_equal(m, np.eye(3)[:2].reshape(-1))
    assert fl == 2


def _tree(root, sub, frames):
    from PIL import Image
    d = os.path.join(root, sub, "frames")
    os.makedirs(d)
    for i, f in enumerate(frames):
        Image.fromarray(f).save(os.path.join(d, f"{i:03d}.png"))


def test_directory_iterator_listing_and_pairing(tmp_path, capsys):
    rng = np.random.default_rng(1)
    sdr = rng.integers(0, 256, (5, 16, 12, 3), dtype=np.uint8)
    hdr = rng.integers(0, 256, (5, 16, 12, 3), dtype=np.uint8)
    _tree(str(tmp_path), "input1", sdr)
    _tree(str(tmp_path), "output1", hdr)
    gi, gm = D.ImageDataGenerator(**REF_ARGS), D.ImageDataGenerator(**REF_ARGS)
    ci, cm = _Capture(gi), _Capture(gm)
    kw = dict(target_size=(16, 12), color_mode="rgb", class_mode=None, batch_size=2, shuffle=True, seed=1)
    it = zip(gi.flow_from_directory(str(tmp_path / "input1"), **kw),
             gm.flow_from_directory(str(tmp_path / "output1"), **kw))
    for _ in range(4):
        next(it)
    assert "Found 5 images belonging to 1 classes." in capsys.readouterr().out
    for (fa, pa), (fb, pb) in zip(ci.seen, cm.seen):
        ia = [int(np.argmax([np.array_equal(f, s) for s in sdr])) for f in fa]
        ib = [int(np.argmax([np.array_equal(f, s) for s in hdr])) for f in fb]
        assert ia == ib and pa == pb  # same frames, same transforms: the pairs stay aligned


def test_resize_nearest_on_load(tmp_path):
    from PIL import Image
    f = np.arange(6 * 4 * 3, dtype=np.uint8).reshape(6, 4, 3)
    p = str(tmp_path / "a.png")
    Image.fromarray(f).save(p)
    a = D.load_img(p, target_size=(3, 2))
    np.testing.assert_array_equal(a, np.asarray(Image.fromarray(f).resize((2, 3), Image.NEAREST)))


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("src_dtype", ["uint8", "float32"])
def test_gpu_warp_matches_scipy(src_dtype):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(3)
    frames = rng.integers(0, 256, (6, 37, 53, 3), dtype=np.uint8)
    if src_dtype == "float32":
        frames = frames.astype(np.float32)
    g = D.ImageDataGenerator(**REF_ARGS)
    r = np.random.RandomState(5)
    params = [g.get_random_transform(f.shape, r) for f in frames]
    params[0].update(theta=0, zx=1, zy=1)  # identity path
    params[1].update(theta=90.0)           # exact quarter turn
    out = g.transform_batch(frames, params).cpu().numpy()
    for i, (f, p) in enumerate(zip(frames, params)):
        ref = A.apply_transform(f.astype(np.float32), p, rescale=1. / 255)
        err = float(np.abs(out[i] - ref).max())
        assert err <= 2e-6, (i, err, p)


@pytest.mark.gpu
def test_gpu_paired_generators_feed_fit_generator(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import contextlib
    import io
    import cnn_itmo_amd as C
    rng = np.random.default_rng(4)
    fr = rng.integers(0, 256, (4, 32, 32, 3), dtype=np.uint8)
    _tree(str(tmp_path), "input1", fr)
    _tree(str(tmp_path), "output1", fr)
    kw = dict(target_size=(32, 32), class_mode=None, batch_size=2, seed=1)
    gen = zip(D.ImageDataGenerator(**REF_ARGS).flow_from_directory(str(tmp_path / "input1"), **kw),
              D.ImageDataGenerator(**REF_ARGS).flow_from_directory(str(tmp_path / "output1"), **kw))
    x, y = next(gen)
    assert x.is_cuda and x.shape == (2, 32, 32, 3)
    assert torch.equal(x, y)  # identical trees -> identical augmented batches
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(32, 32, 3), verbose=False)
    h = m.fit_generator(gen, steps_per_epoch=2, epochs=1, verbose=0)
    assert np.isfinite(h.history["loss"][0])


@pytest.mark.parametrize("world,nfr,bs", [(2, 11, 2), (3, 7, 1), (4, 9, 2)])
def test_rank_shards_union_is_global_stream(world, nfr, bs):
    """8e / 8f row 3: each rank's stream (batch bs) is its contiguous share of the
    single-process stream at batch bs*world -- same frames, same random transforms,
    ragged last batches split as evenly as possible, and a tail with fewer frames
    than ranks (world 4, 9 frames: 8 + 1) dropped on every rank, never an empty share."""
    rng = np.random.default_rng(1)
    frames = rng.integers(0, 256, (nfr, 8, 8, 3), dtype=np.uint8)
    nb = 7
    g = D.ImageDataGenerator(**REF_ARGS)
    cap = _Capture(g)
    it = g.flow(frames, batch_size=bs * world, seed=5, world=1)
    ref, gsz = [], []
    while len(ref) < nb:
        next(it)
        if len(cap.seen[-1][0]) >= world:
            ref.append(cap.seen[-1])
            gsz.append(len(cap.seen[-1][0]))
    shards = []
    for r in range(world):
        gr = D.ImageDataGenerator(**REF_ARGS)
        cr = _Capture(gr)
        itr = gr.flow(frames, batch_size=bs, seed=5, rank=r, world=world)
        assert len(itr) == nfr // (bs * world) + (1 if nfr % (bs * world) >= world else 0)
        for b in range(nb):
            next(itr)
            assert itr.last_global_batch == gsz[b]
        shards.append(cr.seen)
    for b in range(nb):
        fr, params = ref[b]
        got_fr = np.concatenate([shards[r][b][0] for r in range(world)])
        got_p = sum((shards[r][b][1] for r in range(world)), [])
        np.testing.assert_array_equal(got_fr, fr)
        assert got_p == params
        sizes = [len(shards[r][b][0]) for r in range(world)]
        assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1


def test_rank_shards_stay_paired_and_validate():
    """Two generators with the same seed zip into pairs on every rank (main.py:99)."""
    rng = np.random.default_rng(2)
    frames = rng.integers(0, 256, (6, 8, 8, 3), dtype=np.uint8)
    for r in range(2):
        ga, gb = D.ImageDataGenerator(**REF_ARGS), D.ImageDataGenerator(**REF_ARGS)
        ca, cb = _Capture(ga), _Capture(gb)
        ia = ga.flow(frames, batch_size=2, seed=1, rank=r, world=2)
        ib = gb.flow(frames, batch_size=2, seed=1, rank=r, world=2)
        for _ in range(4):
            next(ia), next(ib)
        for (fa, pa), (fb, pb) in zip(ca.seen, cb.seen):
            np.testing.assert_array_equal(fa, fb)
            assert pa == pb
    with pytest.raises(ValueError):
        D.ImageDataGenerator().flow(frames, batch_size=2, seed=None, rank=0, world=2)
    with pytest.raises(ValueError):
        D.ImageDataGenerator().flow(frames, batch_size=2, seed=1, rank=2, world=2)
    with pytest.raises(ValueError):
        D.ImageDataGenerator().flow(frames[:1], batch_size=2, seed=1, rank=0, world=2)


def test_global_batch_of_zip_and_wrappers():
    """Model.fit_generator's global-batch count (model._global_batch): read from the
    zip's own members when all are rank-sharded iterators that agree (main.py:99's
    zip(input, target)); any other wrapper (a prefetching generator, a zip with a
    foreign member, members that disagree) gets None, never another batch's count."""
    from cnn_itmo_amd.model import _global_batch
    frames = np.zeros((7, 8, 8, 3), np.uint8)

    def flow():
        g = D.ImageDataGenerator()
        _Capture(g)
        return g.flow(frames, batch_size=2, seed=1, rank=0, world=2)
    ia, ib = flow(), flow()
    z = zip(ia, ib)
    sizes = []
    for _ in range(3):
        next(z)
        sizes.append(_global_batch(z))
    assert sizes == [4, 3, 4], sizes  # global batch 4 over 2 ranks; the 7-frame epoch's tail is 3
    assert _global_batch(ia) == 4

    def prefetch(it):
        yield from it
    assert _global_batch(prefetch(zip(flow(), flow()))) is None
    assert _global_batch(zip(ia, iter([(frames, frames)]))) is None
    ic, idd = flow(), flow()
    next(ic)
    next(idd)
    next(idd)
    assert _global_batch(zip(ic, idd)) is None  # 4 vs 3: they disagree
