"""BN-folding parity (engine.py module doc): every consumer of a folded BN
output reads the stored post-ReLU r and folds y = r*s + h itself.  Each test
runs the folded kernels on r and compares with the oracle applied to the
materialised y (fp64, zero padding on y), with the same tolerances as
test_gpu_ops.py: fp32 1e-4, bf16 1.5e-2 of the output scale."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import unet_ref as R  # noqa: E402
from tests.test_gpu_ops import DT, TDT, close, dev, host, rnd  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_itmo_amd import _lib as L
    L.load()


def cu(a):
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float32).cuda()


def affine(rng, c, neg=False):
    s = rng.uniform(0.3, 2.0, c)
    if neg:
        s *= np.where(rng.uniform(size=c) < 0.3, -1.0, 1.0)
    return s.astype(np.float32), rng.standard_normal(c).astype(np.float32)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,H,W", [(32, 32, 8, 12), (64, 128, 5, 7), (96, 64, 1, 6), (32, 64, 6, 1),
                                          (128, 256, 3, 4), (64, 64, 8, 64), (32, 96, 4, 128),
                                          (64, 64, 16, 96), (32, 32, 16, 128)])
def test_conv3x3_folded_fwd_wgrad(dt, cin, cout, H, W):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin * 7 + cout + H)
    N, ld, off = 2, cin + 32, 32  # r lives in a concat slice
    rb = np.maximum(rng.standard_normal((N, H, W, ld)), 0).astype(np.float32)
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    s, h = affine(rng, cin)
    d = DT[dt]
    rr = rnd(rb, dt)[..., off:]
    y = rr * s + h
    zref = R.conv2d_same(y, w.astype(np.float64), b)
    wout = torch.empty(w.size, dtype=TDT[dt], device="cuda")
    bout, border = torch.empty(cout, device="cuda"), torch.empty(cout, 8, device="cuda")
    ops.fold_conv3x3(d, cu(w), cu(b), cu(s), cu(h), cout, cin, wout, bout, border)
    rv = ops.View(dev(rb, dt).reshape(-1), N, H, W, cin, ld, off)
    out = ops.new_view(N, H, W, cout, TDT[dt])
    rows = ops.conv3x3_stat_rows(d, N, H, W, cin, cout)
    stats = torch.zeros(rows, 2, cout, device="cuda")
    ops.conv3x3_fwd(d, rv, wout, bout, out, flags=1 | 2, stats=stats, border=border)
    torch.cuda.synchronize()
    close(host(out.buf).reshape(N, H, W, cout), np.maximum(zref, 0), dt, "folded fwd")
    # weight gradient w.r.t. W from r + the fold correction
    dz = rng.standard_normal((N, H, W, cout)).astype(np.float32)
    dzr = rnd(dz, dt)
    _, dw_ref, db_ref = R.conv2d_same_bwd(y, w.astype(np.float64), dzr, need_dx=False)
    dzt = dev(dz, dt)
    db = cu(dzr.reshape(-1, cout).sum(0))
    brows = ops.border_rows(N)
    bpart = torch.empty(brows, 8, cout, device="cuda")
    ops.border_sums(d, dzt, N, H, W, cout, bpart)
    bsum = torch.empty(8, cout, device="cuda")
    ops.colsum(bpart, brows, 8 * cout, 1, bsum)
    want_b = np.stack([dzr[:, 0].sum((0, 1)), dzr[:, -1].sum((0, 1)), dzr[:, :, 0].sum((0, 1)),
                       dzr[:, :, -1].sum((0, 1)), dzr[:, 0, 0].sum(0), dzr[:, 0, -1].sum(0),
                       dzr[:, -1, 0].sum(0), dzr[:, -1, -1].sum(0)])
    dw = torch.empty(cout, 3, 3, cin, device="cuda")
    ops.conv_wgrad(d, 9, rv, dzt, cout, dw, fold=(cu(s), cu(h), db, bsum))
    torch.cuda.synchronize()
    np.testing.assert_allclose(host(bsum), want_b, rtol=1e-4, atol=1e-3)
    close(host(dw), dw_ref, dt, "folded wgrad")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,H,W", [(64, 32, 3, 5), (128, 64, 4, 4), (512, 256, 2, 3)])
def test_tconv_folded_fwd_wgrad(dt, cin, cout, H, W):
    from cnn_itmo_amd import ops
    from cnn_itmo_amd import _lib as L
    rng = np.random.default_rng(cin + 11)
    N = 2
    r = np.maximum(rng.standard_normal((N, H, W, cin)), 0).astype(np.float32)
    k = (rng.standard_normal((2, 2, cout, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    s, h = affine(rng, cin)
    d = DT[dt]
    y = rnd(r, dt) * s + h
    ref = np.maximum(R.tconv2x2s2(y, k.astype(np.float64), b), 0)
    kout = torch.empty(k.size, dtype=TDT[dt], device="cuda")
    bout = torch.empty(4 * cout, device="cuda")
    ops.fold_tconv(d, cu(k), cu(b), cu(s), cu(h), cout, cin, kout, bout)
    xv = ops.View(dev(r, dt).reshape(-1), N, H, W, cin, cin)
    out = ops.new_view(N, 2 * H, 2 * W, cout, TDT[dt])
    ops.tconv_fwd(d, xv, kout, bout, out, flags=L.RELU | L.BIAS_PER_COL)
    torch.cuda.synchronize()
    close(host(out.buf).reshape(ref.shape), ref, dt, "folded tconv fwd")
    dout = rng.standard_normal((N, 2 * H, 2 * W, cout)).astype(np.float32)
    dor = rnd(dout, dt)
    _, dk_ref, _ = R.tconv2x2s2_bwd(y, k.astype(np.float64), dor)
    par = np.stack([dor[:, i::2, j::2].sum((0, 1, 2)) for i in (0, 1) for j in (0, 1)])
    dk = torch.empty(2, 2, cout, cin, device="cuda")
    ops.tconv_wgrad(d, xv, dev(dout, dt), cout, dk, fold=(cu(s), cu(h), cu(par)))
    torch.cuda.synchronize()
    close(host(dk), dk_ref, dt, "folded tconv wgrad")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_bn_bwd_parity_partials_and_r_view(dt):
    """bn_bwd_apply with CNNITMO_PARITY: per-(h&1, w&1) sums of dz; r read from a view."""
    from cnn_itmo_amd import ops
    from cnn_itmo_amd import _lib as L
    rng = np.random.default_rng(12)
    N, H, W, C, ld, off = 2, 6, 10, 64, 96, 32
    rb = np.maximum(rng.standard_normal((N, H, W, ld)), 0).astype(np.float32)
    dy = rng.standard_normal((N, H, W, C)).astype(np.float32)
    d = DT[dt]
    P = N * H * W
    rv = ops.View(dev(rb, dt).reshape(-1), N, H, W, C, ld, off)
    dyv = ops.View(dev(dy, dt).reshape(-1), N, H, W, C, C)
    rows = ops.bn_bwd_rows(P, C)
    part = torch.empty(rows, 4, C, device="cuda")
    dz = torch.empty(P * C, dtype=TDT[dt], device="cuda")
    ops.bn_bwd_apply(d, dyv, rv, C, None, L.NO_BN | L.PARITY, 0, 0, dz, part)
    db, par = torch.empty(C, device="cuda"), torch.empty(4, C, device="cuda")
    ops.colsum(part, rows, 4 * C, 4, db)
    ops.colsum(part, rows, 4 * C, 1, par)
    dz_ref = rnd(dy, dt) * (rnd(rb, dt)[..., off:] > 0)
    dzr = rnd(dz_ref, dt)
    par_ref = np.stack([dzr[:, i::2, j::2].sum((0, 1, 2)) for i in (0, 1) for j in (0, 1)])
    torch.cuda.synchronize()
    close(host(dz).reshape(dz_ref.shape), dz_ref, dt, "dz")
    np.testing.assert_allclose(host(par), par_ref, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(host(db), par_ref.sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_maxpool_affine(dt):
    """Pool over y = r*s + h with some negative scales (max of y is not max of r)."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(13)
    N, H, W, C, ld, off = 2, 6, 8, 64, 96, 32
    rb = np.maximum(rng.standard_normal((N, H, W, ld)), 0).astype(np.float32)
    s, h = affine(rng, C, neg=True)
    d = DT[dt]
    xv = ops.View(dev(rb, dt).reshape(-1), N, H, W, C, ld, off)
    y = torch.empty(N * H // 2 * W // 2 * C, dtype=TDT[dt], device="cuda")
    idx = torch.empty(N * H // 2 * W // 2 * C, dtype=torch.uint8, device="cuda")
    ops.maxpool_fwd(d, xv, y, idx, aff=(cu(s), cu(h)))
    # the kernel computes y in fp32 from the stored r
    yin = (rnd(rb, dt)[..., off:].astype(np.float32) * s + h).astype(np.float64)
    yr, ir = R.maxpool2x2(yin)
    torch.cuda.synchronize()
    close(host(y).reshape(yr.shape), yr, dt, "pool affine")
    assert np.array_equal(idx.cpu().numpy().reshape(ir.shape), ir)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_head_folded(dt):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(14)
    N, Hv, H, W, C = 2, 7, 8, 16, 64
    r = np.maximum(rng.standard_normal((N, H, W, C)), 0).astype(np.float32)
    w = (rng.standard_normal((3, C)) * 0.2).astype(np.float32)
    b = rng.standard_normal(3).astype(np.float32)
    s, h = affine(rng, C)
    t = rng.uniform(size=(N, Hv, W, 3)).astype(np.float32)
    d = DT[dt]
    xv = ops.View(dev(r, dt).reshape(-1), N, H, W, C, C)
    aff = (cu(s), cu(h))
    yh = torch.empty(N, Hv, W, 3, device="cuda")
    ops.head_fwd(d, xv, Hv, cu(w), cu(b), yh, aff=aff)
    y = (rnd(r, dt) * s + h)[:, :Hv]
    yref = R.sigmoid(y @ w.T.astype(np.float64) + b)
    rows = ops.head_rows(N * H * W)
    part = torch.empty(rows, 5 + 3 * C, device="cuda")
    dx = torch.empty(N * H * W * C, dtype=TDT[dt], device="cuda")
    ops.head_fwd_bwd(d, xv, Hv, cu(w), cu(b), cu(t), dx, part, aff=aff)
    la, dw, db = torch.empty(2, device="cuda"), torch.empty(3, C, device="cuda"), torch.empty(3, device="cuda")
    ops.head_finalize(part, rows, C, N * Hv * W * 3, la, dw, db, aff=aff)
    dz = R.mse_grad_z(yref, t)
    dx_ref = np.zeros((N, H, W, C))
    dx_ref[:, :Hv] = dz @ w.astype(np.float64)
    torch.cuda.synchronize()
    close(yh.cpu().numpy(), yref, "f32", "yhat")
    assert abs(la[0].item() - R.mse(yref, t)) < 1e-5
    close(host(dw) * 1e3, dz.reshape(-1, 3).T @ y.reshape(-1, C) * 1e3, "f32", "head dw")
    close(host(db) * 1e3, dz.reshape(-1, 3).sum(0) * 1e3, "f32", "head db")
    close(host(dx).reshape(dx_ref.shape) * 1e3, dx_ref * 1e3, dt, "head dx")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("H,W", [(6, 10), (7, 9)])
def test_pool_deferred_route_and_sums(dt, H, W):
    """A pooled folded BN output: the pool's share of the BN-backward sums
    (cnnitmo_pool_bnsums) and the BN apply with the pool routing folded in
    (cnnitmo_bn_bwd_apply_pooled) == maxpool_bwd followed by bn_bwd_apply."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(14)
    N, C, ld, off = 2, 64, 96, 32
    Ho, Wo = H // 2, W // 2
    d = DT[dt]
    rb = np.maximum(rng.standard_normal((N, H, W, ld)), 0).astype(np.float32)
    dy = rng.standard_normal((N, H, W, C)).astype(np.float32)
    dyp = rng.standard_normal((N, Ho, Wo, C)).astype(np.float32)
    idx = rng.integers(0, 4, (N, Ho, Wo, C)).astype(np.uint8)
    mean = rng.uniform(0.2, 0.8, C).astype(np.float32)
    inv = rng.uniform(0.5, 2.0, C).astype(np.float32)
    coef = rng.standard_normal(3 * C).astype(np.float32)
    P = N * H * W
    rv = ops.View(dev(rb, dt).reshape(-1), N, H, W, C, ld, off)
    dyp_t, idx_t = dev(dyp, dt).reshape(-1), torch.tensor(idx.reshape(-1)).cuda()

    rows = ops.bn_bwd_rows(N * Ho * Wo, C)
    pm = torch.empty(rows, 2, C, device="cuda")
    ops.pool_bnsums(d, dyp_t, idx_t, rv, cu(mean), cu(inv), pm)
    sums = torch.empty(2, C, device="cuda")
    ops.colsum(pm, rows, 2 * C, 1, sums)
    r64 = rnd(rb, dt)[..., off:].astype(np.float64)
    g64 = rnd(dyp, dt).astype(np.float64)
    rwin = r64[:, :2 * Ho, :2 * Wo].reshape(N, Ho, 2, Wo, 2, C).transpose(0, 1, 3, 2, 4, 5).reshape(N, Ho, Wo, 4, C)
    rarg = np.take_along_axis(rwin, idx[:, :, :, None, :].astype(np.int64), axis=3)[:, :, :, 0]
    want = np.stack([g64.sum((0, 1, 2)), (g64 * (rarg - mean) * inv).sum((0, 1, 2))])
    torch.cuda.synchronize()
    np.testing.assert_allclose(host(sums), want, rtol=1e-4, atol=1e-3)

    rows2 = ops.bn_bwd_rows(P, C)
    dy_a = dev(dy, dt).reshape(-1)
    dz_a = torch.empty(P * C, dtype=TDT[dt], device="cuda")
    pa = torch.empty(rows2, C, device="cuda")
    ops.bn_bwd_apply_pooled(d, ops.View(dy_a, N, H, W, C, C), rv, C, cu(coef), dyp_t, idx_t, dz_a, pa)
    dy_b = dev(dy, dt).reshape(-1)
    ops.maxpool_bwd(d, dyp_t, idx_t, ops.View(dy_b, N, H, W, C, C))
    dz_b = torch.empty(P * C, dtype=TDT[dt], device="cuda")
    pb = torch.empty(rows2, C, device="cuda")
    ops.bn_bwd_apply(d, ops.View(dy_b, N, H, W, C, C), rv, C, cu(coef), 0, 0, 0, dz_b, pb)
    db_a, db_b = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.colsum(pa, rows2, C, 1, db_a)
    ops.colsum(pb, rows2, C, 1, db_b)
    torch.cuda.synchronize()
    # bf16: the reference path rounds dy + routed to bf16 before the apply
    tol = 1e-5 if dt == "f32" else 2e-2
    np.testing.assert_allclose(host(dz_a), host(dz_b), rtol=tol, atol=tol * 4)
    np.testing.assert_allclose(host(db_a), host(db_b), rtol=tol, atol=tol * 20)


@pytest.mark.parametrize("cin,cout,H,W,c0,c1,par", [
    (32, 32, 20, 40, 0, 32, False),      # the whole input (enc1a -> enc1b), partial tiles
    (96, 64, 18, 70, 32, 96, True),      # concat [skip 32 | up 64] -> BN 48 blocks (6 of 8 lanes)
    (160, 64, 16, 40, 32, 160, True),    # BN 32 blocks
    (192, 128, 16, 32, 64, 192, True),   # concat [skip 64 | up 128] -> BN 64 blocks
    (128, 64, 17, 33, 0, 128, False)])
@pytest.mark.parametrize("dt", ["bf16", "f32"])
def test_conv3x3_dgrad_bn_fused(cin, cout, H, W, c0, c1, par, dt):
    """cnnitmo_conv3x3_dgrad_bn == conv3x3_dgrad followed by bn_bwd_apply on the
    fused column range (same coefficients, r read from a concat-style view);
    columns outside the range are the plain input gradient.  fp32: the halo kernel's
    fp32 fused epilogue (fp32 training, 16-channel chunks)."""
    from cnn_itmo_amd import ops
    from cnn_itmo_amd import _lib as L
    rng = np.random.default_rng(cin + c0 + H)
    N, d, c = 2, DT[dt], c1 - c0
    T = TDT[dt]
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    wf = torch.empty(w.size, dtype=T, device="cuda")
    wflip = torch.empty(w.size, dtype=T, device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cin, wf, wflip)
    dz = dev(rng.standard_normal((N, H, W, cout)).astype(np.float32), dt).reshape(-1)
    rb = dev(np.maximum(rng.standard_normal((N, H, W, cin)), 0).astype(np.float32), dt).reshape(-1)
    rv = ops.View(rb, N, H, W, c, cin, c0)
    coef = cu(rng.standard_normal(3 * c).astype(np.float32))
    P = N * H * W
    # unfused reference path
    g = torch.zeros(P * cin, dtype=T, device="cuda")
    ops.conv3x3_dgrad(d, dz, N, H, W, cout, wflip, cin, ops.View(g, N, H, W, cin, cin, 0))
    rows = ops.bn_bwd_rows(P, c)
    np_ = 4 if par else 1
    pref = torch.empty(rows * np_ * c, device="cuda")
    zref = torch.empty(P * c, dtype=T, device="cuda")
    ops.bn_bwd_apply(d, ops.View(g, N, H, W, c, cin, c0), rv, c, coef, L.PARITY if par else 0, 0, 0, zref, pref)
    sref = torch.empty(np_ * c, device="cuda")
    ops.colsum(pref, rows, np_ * c, 1, sref)
    # fused
    frows = ops.conv3x3_dgrad_bn_rows(d, N, H, W, cout, cin, c0, c1)
    assert frows > 0
    whole = c0 == 0 and c1 == cin
    dx = None if whole else ops.View(torch.zeros(P * cin, dtype=T, device="cuda"), N, H, W, cin, cin)
    zf = torch.empty(P * c, dtype=T, device="cuda")
    pf = torch.empty(frows * np_ * c, device="cuda")
    ops.conv3x3_dgrad_bn(d, dz, N, H, W, cout, wflip, cin, dx, c0, c1, coef, rv, zf, pf, par)
    sf = torch.empty(np_ * c, device="cuda")
    ops.colsum(pf, frows, np_ * c, 1, sf)
    torch.cuda.synchronize()
    a, b = host(zf), host(zref)
    if dt == "f32":  # the same fp32 g and formula (up to an fma contraction)
        assert np.abs(a - b).max() <= 1e-5 * max(1.0, np.abs(b).max())
    else:  # same bf16 g and formula; an fp32 contraction difference may flip one bf16 rounding
        assert np.abs(a - b).max() <= 1e-2 * max(1.0, np.abs(b).max())
        assert np.mean(a != b) < 1e-3
    np.testing.assert_allclose(host(sf), host(sref), rtol=1e-4, atol=1e-2)
    if not whole:
        gx = host(dx.buf).reshape(P, cin)
        gr = host(g).reshape(P, cin)
        assert np.array_equal(gx[:, :c0], gr[:, :c0]) and np.array_equal(gx[:, c1:], gr[:, c1:])
        assert float(np.abs(gx[:, c0:c1]).max()) == 0.0  # fused columns are not written to dx


@pytest.mark.parametrize("cin,cout,H,W", [
    (32, 64, 20, 40),     # dec9's skip path (conv1 32 of the [32 | 64] concat), partial tiles
    (32, 64, 34, 70),     # ragged in both directions (partial 16-row tiles, 32-column strips)
    (64, 128, 16, 32),    # BN 64 (a level-1 skip path)
    (32, 96, 18, 66)])
@pytest.mark.parametrize("dt", ["bf16", "f32"])
def test_conv3x3_dgrad_bn_pooled(cin, cout, H, W, dt):
    """cnnitmo_conv3x3_dgrad_bn_pooled == conv3x3_dgrad of the skip rows, then
    bn_bwd_apply_pooled (the pooled gradient routed by the window index bytes) with
    the same coefficients: the deferred skip gradient of dec9 fused with conv1's
    MaxPooling2D route and BN backward."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin + cout + H + W)
    N, d = 2, DT[dt]
    T = TDT[dt]
    cl = cin + 64  # the concat consumer's input channels: skip rows [0, cin) of its flipped weights
    w = (rng.standard_normal((cout, 3, 3, cl)) * 0.1).astype(np.float32)
    wf = torch.empty(w.size, dtype=T, device="cuda")
    wflip = torch.empty(w.size, dtype=T, device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cl, wf, wflip)
    dz = dev(rng.standard_normal((N, H, W, cout)).astype(np.float32), dt).reshape(-1)
    rb = dev(np.maximum(rng.standard_normal((N, H, W, cin)), 0).astype(np.float32), dt).reshape(-1)
    rv = ops.View(rb, N, H, W, cin, cin, 0)
    dyp = dev(rng.standard_normal((N, H // 2, W // 2, cin)).astype(np.float32), dt).reshape(-1)
    idx = torch.tensor(rng.integers(0, 4, (N, H // 2, W // 2, cin)).astype(np.uint8).reshape(-1)).cuda()
    coef = cu(rng.standard_normal(3 * cin).astype(np.float32))
    P = N * H * W
    # unfused reference path: the skip gradient stored, then the pooled BN-backward apply
    g = torch.zeros(P * cin, dtype=T, device="cuda")
    gv = ops.View(g, N, H, W, cin, cin, 0)
    ops.conv3x3_dgrad(d, dz, N, H, W, cout, wflip, cin, gv)
    rows = ops.bn_bwd_rows(P, cin)
    pref = torch.empty(rows * cin, device="cuda")
    zref = torch.empty(P * cin, dtype=T, device="cuda")
    ops.bn_bwd_apply_pooled(d, gv, rv, cin, coef, dyp, idx, zref, pref)
    sref = torch.empty(cin, device="cuda")
    ops.colsum(pref, rows, cin, 1, sref)
    # fused
    frows = ops.conv3x3_dgrad_bn_pooled_rows(d, N, H, W, cout, cin)
    assert frows > 0
    zf = torch.full((P * cin,), float("nan"), dtype=T, device="cuda")
    pf = torch.empty(frows * cin, device="cuda")
    ops.conv3x3_dgrad_bn_pooled(d, dz, N, H, W, cout, wflip, cin, coef, rv, dyp, idx, zf, pf)
    sf = torch.empty(cin, device="cuda")
    ops.colsum(pf, frows, cin, 1, sf)
    torch.cuda.synchronize()
    a, b = host(zf), host(zref)
    assert np.isfinite(a).all()
    if dt == "f32":  # the same fp32 g and formula (up to an fma contraction)
        assert np.abs(a - b).max() <= 1e-5 * max(1.0, np.abs(b).max())
    else:  # the same bf16-rounded g; an fp32 contraction difference may flip one bf16 rounding
        assert np.abs(a - b).max() <= 1e-2 * max(1.0, np.abs(b).max())
        assert np.mean(a != b) < 1e-3
    np.testing.assert_allclose(host(sf), host(sref), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("cin,cout,H,W", [(128, 64, 3, 70), (64, 32, 4, 64), (128, 32, 2, 130)])
def test_tconv_dgrad_bn_fused(cin, cout, H, W):
    """cnnitmo_tconv2x2_dgrad_bn == tconv2x2_dgrad followed by bn_bwd_apply (r from a view)."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin + W)
    N, d = 2, DT["bf16"]
    k = (rng.standard_normal((2, 2, cout, cin)) * 0.1).astype(np.float32)
    kf = torch.empty(k.size, dtype=torch.bfloat16, device="cuda")
    kT = torch.empty(k.size, dtype=torch.bfloat16, device="cuda")
    ops.prep_tconv(d, torch.tensor(k).cuda(), cout, cin, kf, kT)
    dout = dev(rng.standard_normal((N, 2 * H, 2 * W, cout)).astype(np.float32), "bf16").reshape(-1)
    ld, off = cin + 32, 32
    rb = dev(np.maximum(rng.standard_normal((N, H, W, ld)), 0).astype(np.float32), "bf16").reshape(-1)
    rv = ops.View(rb, N, H, W, cin, ld, off)
    coef = cu(rng.standard_normal(3 * cin).astype(np.float32))
    P = N * H * W
    g = torch.empty(P * cin, dtype=torch.bfloat16, device="cuda")
    ops.tconv_dgrad(d, dout, N, H, W, cout, kT, cin, g)
    rows = ops.bn_bwd_rows(P, cin)
    pref = torch.empty(rows * cin, device="cuda")
    zref = torch.empty(P * cin, dtype=torch.bfloat16, device="cuda")
    ops.bn_bwd_apply(d, ops.View(g, N, H, W, cin, cin), rv, cin, coef, 0, 0, 0, zref, pref)
    sref = torch.empty(cin, device="cuda")
    ops.colsum(pref, rows, cin, 1, sref)
    frows = ops.tconv_dgrad_bn_rows(d, N, H, W, cout, cin)
    assert frows > 0
    zf = torch.empty(P * cin, dtype=torch.bfloat16, device="cuda")
    pf = torch.empty(frows * cin, device="cuda")
    ops.tconv_dgrad_bn(d, dout, N, H, W, cout, kT, cin, coef, rv, zf, pf)
    sf = torch.empty(cin, device="cuda")
    ops.colsum(pf, frows, cin, 1, sf)
    torch.cuda.synchronize()
    a, b = host(zf), host(zref)
    assert np.abs(a - b).max() <= 1e-2 * max(1.0, np.abs(b).max())
    assert np.mean(a != b) < 1e-3
    np.testing.assert_allclose(host(sf), host(sref), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("kind,cin,cout,H,W,c0,c1", [
    ("c3", 96, 64, 18, 70, 32, 96),     # dec9-style concat [skip 32 | up 64]
    ("c3", 64, 64, 16, 64, 0, 64),      # whole input (enc chain)
    ("c3", 192, 128, 16, 32, 64, 192),  # dec8-style
    ("t2", 128, 64, 3, 70, 0, 128)])    # up9 dgrad into conv8's BN
def test_dgrad_bn_fused_vs_oracle(kind, cin, cout, H, W, c0, c1):
    """The fused dgrad + producer-BN-backward pinned DIRECTLY to the oracle:
    R.conv2d_same_bwd / R.tconv2x2s2_bwd for g, then R.bn_train_bwd and the ReLU
    mask for the producer's dz.  Coefficients come from the product's
    cnnitmo_bn_bwd_finalize fed the oracle's sums (sum dy, sum dy*rhat)."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin + cout + H)
    N, d, c = 2, DT["bf16"], c1 - c0
    ho, wo = (H, W) if kind == "c3" else (2 * H, 2 * W)
    if kind == "c3":
        w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    else:
        w = (rng.standard_normal((2, 2, cout, cin)) * 0.1).astype(np.float32)
    wr = rnd(w, "bf16")
    wf = torch.empty(w.size, dtype=torch.bfloat16, device="cuda")
    wb = torch.empty(w.size, dtype=torch.bfloat16, device="cuda")
    (ops.prep_conv3x3 if kind == "c3" else ops.prep_tconv)(d, torch.tensor(w).cuda(), cout, cin, wf, wb)
    dz = rnd(rng.standard_normal((N, ho, wo, cout)), "bf16")
    r = rnd(np.maximum(rng.standard_normal((N, H, W, c)) + 0.3, 0), "bf16")  # producer post-ReLU
    gamma = rng.uniform(0.5, 1.5, c)
    mean, var = r.reshape(-1, c).mean(0), r.reshape(-1, c).var(0)
    inv = 1.0 / np.sqrt(var + R.BN_EPS)
    # oracle: consumer input gradient, producer BN backward, ReLU mask
    if kind == "c3":
        g = R.conv2d_same_bwd(np.zeros((N, H, W, cin)), wr, dz)[0]
    else:
        g = R.tconv2x2s2_bwd(np.zeros((N, H, W, cin)), wr, dz)[0]
    dy = rnd(g[..., c0:c1], "bf16")  # the fused store applies the BN backward to bf16(g)
    dr, dgam, dbet = R.bn_train_bwd(dy, r, gamma, mean, var)
    want = dr * (r > 0)
    # product: finalize on the oracle's sums -> coef, then the fused kernel
    rhat = (r - mean) * inv
    part = np.stack([dy.reshape(-1, c).sum(0), (dy * rhat).reshape(-1, c).sum(0)])[None]  # [1][2][c]
    coef = torch.empty(3 * c, device="cuda")
    dgg, dbb = torch.empty(c, device="cuda"), torch.empty(c, device="cuda")
    ops.bn_bwd_finalize(cu(part.astype(np.float32)), 1, c, N * H * W, cu(gamma.astype(np.float32)),
                        cu(mean.astype(np.float32)), cu(inv.astype(np.float32)), dgg, dbb, coef)
    rv = dev(r, "bf16").reshape(-1)
    zf = torch.empty(N * H * W * c, dtype=torch.bfloat16, device="cuda")
    dzd = dev(dz, "bf16").reshape(-1)
    if kind == "c3":
        frows = ops.conv3x3_dgrad_bn_rows(d, N, H, W, cout, cin, c0, c1)
        whole = c0 == 0 and c1 == cin
        dx = None if whole else ops.View(torch.zeros(N * H * W * cin, dtype=torch.bfloat16, device="cuda"),
                                         N, H, W, cin, cin)
        pf = torch.empty(frows * c, device="cuda")
        ops.conv3x3_dgrad_bn(d, dzd, N, H, W, cout, wb, cin, dx, c0, c1, coef, rv, zf, pf, False)
    else:
        frows = ops.tconv_dgrad_bn_rows(d, N, H, W, cout, cin)
        pf = torch.empty(frows * c, device="cuda")
        ops.tconv_dgrad_bn(d, dzd, N, H, W, cout, wb, cin, coef, rv, zf, pf)
    torch.cuda.synchronize()
    np.testing.assert_allclose(host(dgg), dgam, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(host(dbb), dbet, rtol=1e-5, atol=1e-5)
    got = host(zf).reshape(want.shape)
    # bf16 store of an fp32 evaluation (+ one bf16 ulp of g that may round differently)
    bound = 2.0 ** -8 * np.abs(want) + 2.0 ** -7 * np.abs(gamma * inv * dy) + 1e-3 * np.abs(want).max()
    assert float((np.abs(got - want) / bound).max()) <= 1.0
    if kind == "c3" and not (c0 == 0 and c1 == cin):
        gx = host(dx.buf).reshape(N, H, W, cin)
        np.testing.assert_allclose(gx[..., :c0], g[..., :c0], rtol=2 ** -7, atol=1e-2 * np.abs(g).max())
