"""Tone-mapping maps: cnn_itmo_amd/tonemap.py + csrc/tonemap.hip
vs oracle/tonemap_ref.py (a float64 restatement of m-files/Reinhard.m,
virtual_camera.m and inverse_Reinhard.m; RGB2Lum is not in the reference, so
the Rec. 709 weights are a stated choice -- parity unpinned for it).

Tolerances: float32 outputs rtol 2e-6 (float64 arithmetic on both sides; the
last bits of log/exp/pow and the summation order differ); uint8 outputs (imwrite
uint8(255*x)) may differ by 1 LSB only where 255*x sits on a .5 tie, < 0.1 %.
Property at full size: inverse_reinhard(reinhard(hdr), g=G, 'exact') == hdr."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import tonemap_ref as T  # noqa: E402


def _hdr(rng, n, h, w):
    return np.exp(rng.normal(-1.0, 1.5, (n, h, w, 3))).astype(np.float32)


# --------------------------------------------------------------------- CPU (oracle)
def test_oracle_reinhard_constant_image():
    hdr = np.full((4, 5, 3), 2.0, np.float32)
    sdr = T.reinhard(hdr)
    # Y = 2 everywhere -> G = 2 -> X = 0.18 -> L = 0.18/1.18 -> sdr = 2 * L / 2
    np.testing.assert_allclose(sdr, 0.18 / 1.18, rtol=1e-15)


def test_oracle_matlab_semantics():
    assert T.im2uint8(np.array([np.nan, -1, 0.5 / 255, 1.5 / 255, 2.0]))[0] == 0
    np.testing.assert_array_equal(T.im2uint8(np.array([np.nan, -1, 0.5 / 255, 1.5 / 255, 2.0])),
                                  [0, 0, 1, 2, 255])
    hdr = np.zeros((2, 2, 3), np.float32)
    hdr[0, 0] = 1.0
    out = T.reinhard(hdr)  # zero-luminance pixels: 0/0 -> NaN, as in MATLAB
    assert np.isnan(out[1, 1]).all() and np.isfinite(out[0, 0]).all()
    vc = T.virtual_camera(hdr, 0.0, 0.6, -0.5)  # X^y = inf at X = 0 -> NaN -> min(1, NaN) = 1
    assert np.isfinite(vc[0, 0]).all()


def test_oracle_exact_inverse_roundtrip():
    rng = np.random.default_rng(0)
    hdr = _hdr(rng, 1, 8, 9)[0].astype(np.float64)
    G = T.log_average(T.rgb2lum(hdr))
    back = T.inverse_reinhard(T.reinhard(hdr), mode="exact", g=G)
    np.testing.assert_allclose(back, hdr, rtol=1e-9)


# ------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_itmo_amd import tonemap
    return tonemap


@pytest.mark.gpu
def test_gpu_reinhard_matches_oracle(gpu):
    rng = np.random.default_rng(1)
    hdr = _hdr(rng, 3, 37, 61)
    hdr[0, 0, 0] = 0.0  # a zero-luminance pixel: NaN like MATLAB
    out = gpu.reinhard(hdr).cpu().numpy()
    for i in range(3):
        ref = T.reinhard(hdr[i]).astype(np.float32)
        np.testing.assert_allclose(out[i], ref, rtol=2e-6, atol=0, equal_nan=True)
    G = gpu.log_average(hdr).cpu().numpy()
    for i in range(3):
        np.testing.assert_allclose(G[i], T.log_average(T.rgb2lum(hdr[i])), rtol=1e-12)
    u8 = gpu.reinhard(hdr, out_u8=True).cpu().numpy().astype(int)
    ref8 = np.stack([T.im2uint8(T.reinhard(h)) for h in hdr]).astype(int)
    d = np.abs(u8 - ref8)
    assert d.max() <= 1 and (d > 0).mean() < 1e-3


@pytest.mark.gpu
def test_gpu_virtual_camera_matches_oracle(gpu):
    rng = np.random.default_rng(2)
    hdr = _hdr(rng, 4, 33, 40)
    v, n, y = gpu.virtual_camera_params(4, np.random.default_rng(3))
    out = gpu.virtual_camera(hdr, v, n, y).cpu().numpy()
    for i in range(4):
        ref = T.virtual_camera(hdr[i], v[i], n[i], y[i]).astype(np.float32)
        np.testing.assert_allclose(out[i], ref, rtol=2e-6, atol=1e-30, equal_nan=True)


@pytest.mark.gpu
def test_gpu_inverse_script_matches_oracle(gpu):
    rng = np.random.default_rng(4)
    sdr = rng.integers(0, 256, (2, 20, 30, 3), dtype=np.uint8)
    sdr[1, :2] = 0  # some zero-luminance pixels: PB1 > 0
    out = gpu.inverse_reinhard(sdr, mode="script").cpu().numpy()
    for i in range(2):
        ref = T.inverse_reinhard(sdr[i], mode="script").astype(np.float32)
        np.testing.assert_allclose(out[i], ref, rtol=2e-6, atol=1e-37, equal_nan=True)


@pytest.mark.gpu
def test_gpu_exact_roundtrip_full_hd(gpu):
    """Size-independent property at 1080p: the exact inverse undoes Reinhard."""
    rng = np.random.default_rng(5)
    hdr = _hdr(rng, 2, 1080, 1920)
    sdr = gpu.reinhard(hdr)
    G = gpu.log_average(hdr).cpu().numpy()
    for i in range(2):
        back = gpu.inverse_reinhard(sdr[i:i + 1], mode="exact", g=float(G[i]))[0].cpu().numpy()
        # the fp32 SDR in between limits it: X = L/(1-L) amplifies L's rounding by 1/(1-L)
        np.testing.assert_allclose(back, hdr[i], rtol=3e-5)
