"""Per-kernel parity: every C-ABI entry point vs the numpy oracle (fp64) on the
same seeded inputs.  fp32 path: max-abs <= 1e-4 relative to the output scale
(MFMA f32 is an exact fp32 fma chain).  bf16 path: inputs are rounded to bf16
first and the oracle sees the same rounded values; tolerance 1.5e-2 of scale
(bf16 output rounding is 2^-8)."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import unet_ref as R  # noqa: E402

DT = {"f32": 0, "bf16": 1}
TDT = {"f32": torch.float32, "bf16": torch.bfloat16}
TOL = {"f32": 1e-4, "bf16": 1.5e-2}


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_itmo_amd import _lib as L
    L.load()


def dev(a, dt):
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float32).to(TDT[dt]).cuda()


def rnd(a, dt):
    """Round host array through the device dtype (what the kernel actually sees)."""
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float32).to(TDT[dt]).double().numpy()


def host(t):
    return t.float().cpu().numpy().astype(np.float64)


def close(got, want, dt, what=""):
    scale = max(1.0, float(np.abs(want).max()))
    err = float(np.abs(got - want).max())
    assert err <= TOL[dt] * scale, f"{what}: max-abs err {err:.3e} > {TOL[dt] * scale:.3e}"


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,H,W", [(32, 32, 8, 12), (64, 128, 5, 7), (96, 64, 6, 10), (32, 256, 4, 4),
                                          # whole 4x64 tiles: the halo kernel (bf16) for fwd and dgrad
                                          (32, 32, 8, 64), (96, 64, 4, 128), (192, 128, 4, 64),
                                          (64, 64, 12, 64), (32, 64, 12, 192), (96, 64, 16, 128),
                                          (192, 128, 8, 64), (64, 64, 16, 64), (32, 64, 24, 192),
                                          # 128-channel-deep wgrad blocks, a partial last strip
                                          (128, 64, 6, 64), (256, 128, 10, 70)])
def test_conv3x3_fwd_dgrad_wgrad(dt, cin, cout, H, W):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin + cout)
    N = 2
    # input lives in a wider buffer (zero-copy concat view): ld = cin + 32, off = 32
    ld, off = cin + 32, 32
    xb = rng.standard_normal((N, H, W, ld)).astype(np.float32)
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    x = rnd(xb, dt)[..., off:]
    wr = rnd(w, dt)
    z = R.conv2d_same(x, wr, b)
    r_ref = np.maximum(z, 0)
    xbuf = dev(xb, dt).reshape(-1)
    xv = ops.View(xbuf, N, H, W, cin, ld, off)
    d = DT[dt]
    wf = torch.empty(w.size, dtype=TDT[dt], device="cuda")
    wflip = torch.empty(w.size, dtype=TDT[dt], device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cin, wf, wflip)
    out = ops.new_view(N, H, W, cout, TDT[dt])
    rows = ops.conv3x3_stat_rows(d, N, H, W, cin, cout)
    stats = torch.zeros(rows, 2, cout, device="cuda")
    ops.conv3x3_fwd(d, xv, wf, torch.tensor(b).cuda(), out, flags=1 | 2, stats=stats)
    torch.cuda.synchronize()
    close(host(out.buf).reshape(N, H, W, cout), r_ref, dt, "fwd")
    s = stats.sum(0).double().cpu().numpy()
    close(s[0] / r_ref.size * cout, r_ref.reshape(-1, cout).mean(0), dt, "stat sum")
    # dgrad into a view of a wider buffer
    dz = rng.standard_normal((N, H, W, cout)).astype(np.float32)
    dzr = rnd(dz, dt)
    dx_ref, dw_ref, db_ref = R.conv2d_same_bwd(x, wr, dzr)
    dxb = torch.zeros(N * H * W * ld, dtype=TDT[dt], device="cuda")
    ops.conv3x3_dgrad(d, dev(dz, dt), N, H, W, cout, wflip, cin, ops.View(dxb, N, H, W, cin, ld, off))
    torch.cuda.synchronize()
    close(host(dxb).reshape(N, H, W, ld)[..., off:], dx_ref, dt, "dgrad")
    assert float(host(dxb).reshape(N, H, W, ld)[..., :off].max()) == 0.0  # other slice untouched
    dw = torch.empty(cout, 3, 3, cin, device="cuda")
    ops.conv_wgrad(d, 9, xv, dev(dz, dt), cout, dw)
    torch.cuda.synchronize()
    close(host(dw), dw_ref, dt, "wgrad")


def test_conv3x3_halo_tall_frame():
    """Halo kernel on a frame taller than 1024 rows (tile row offsets > 1000), bf16."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(21)
    N, H, W, cin, cout = 1, 1032, 128, 32, 32
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    d = DT["bf16"]
    wf = torch.empty(w.size, dtype=TDT["bf16"], device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cin, wf, None)
    out = ops.new_view(N, H, W, cout, TDT["bf16"])
    ops.conv3x3_fwd(d, ops.View(dev(x, "bf16").reshape(-1), N, H, W, cin, cin), wf, torch.tensor(b).cuda(),
                    out, flags=1)
    ref = np.maximum(R.conv2d_same(rnd(x, "bf16"), rnd(w, "bf16"), b), 0)
    torch.cuda.synchronize()
    close(host(out.buf).reshape(ref.shape), ref, "bf16", "tall frame")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("H,W", [(6, 9), (4, 64)])
def test_conv_affine_inference_epilogue(dt, H, W):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(3)
    N, cin, cout = 1, 32, 64
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    sc = rng.uniform(0.5, 2, cout).astype(np.float32)
    sh = rng.standard_normal(cout).astype(np.float32)
    d = DT[dt]
    wf = torch.empty(w.size, dtype=TDT[dt], device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cin, wf, None)
    out = ops.new_view(N, H, W, cout, TDT[dt])
    ops.conv3x3_fwd(d, ops.View(dev(x, dt).reshape(-1), N, H, W, cin, cin), wf, torch.tensor(b).cuda(), out,
                    flags=1 | 4, aff=(torch.tensor(sc).cuda(), torch.tensor(sh).cuda()))
    ref = np.maximum(R.conv2d_same(rnd(x, dt), rnd(w, dt), b), 0) * sc + sh
    torch.cuda.synchronize()
    close(host(out.buf).reshape(ref.shape), ref, dt, "affine")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,H,W", [(64, 32, 3, 5), (128, 64, 4, 4), (512, 256, 2, 3),
                                          # bf16: the streamed kernel (resident weights), partial 64-px tiles
                                          (128, 64, 3, 70), (256, 128, 5, 33), (128, 32, 2, 130),
                                          # bf16 weight-stationary kernel: fwd at 32 column blocks
                                          # (512 -> 512), dgrad at BN 128 (256 <- 128); ragged tiles
                                          (512, 512, 3, 7), (256, 128, 7, 9),
                                          # 1024 / 2048-deep gradients (up7 / up6: igemm_fwd2p's
                                          # persistent 256 x 256 tiles; ragged tiles)
                                          (512, 256, 5, 7), (512, 256, 17, 33), (256, 512, 9, 31),
                                          # > 256 tiles of 256 x 256: each persistent workgroup
                                          # (igemm_fwd2p_kernel, one per CU) walks several
                                          (512, 256, 96, 176),
                                          # bf16 row-streaming wgrad: 4 rows per workgroup, 2 strips
                                          (512, 512, 16, 40)])
def test_tconv(dt, cin, cout, H, W):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin)
    N = 2
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    k = (rng.standard_normal((2, 2, cout, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    d = DT[dt]
    xr, kr = rnd(x, dt), rnd(k, dt)
    ref = np.maximum(R.tconv2x2s2(xr, kr, b), 0)
    kf = torch.empty(k.size, dtype=TDT[dt], device="cuda")
    kT = torch.empty(k.size, dtype=TDT[dt], device="cuda")
    ops.prep_tconv(d, torch.tensor(k).cuda(), cout, cin, kf, kT)
    # output into a concat slice: ld = cout + 64, off = 64
    ld = cout + 64
    ob = torch.zeros(N * 2 * H * 2 * W * ld, dtype=TDT[dt], device="cuda")
    rows = ops.tconv_stat_rows(d, N, H, W, cin, cout)
    stats = torch.zeros(rows, 2, 4 * cout, device="cuda")
    xv = ops.View(dev(x, dt).reshape(-1), N, H, W, cin, cin)
    ops.tconv_fwd(d, xv, kf, torch.tensor(b).cuda(), ops.View(ob, N, 2 * H, 2 * W, cout, ld, 64),
                  flags=1 | 2, stats=stats)
    torch.cuda.synchronize()
    got = host(ob).reshape(N, 2 * H, 2 * W, ld)
    close(got[..., 64:], ref, dt, "tconv fwd")
    s = stats.sum(0).double().cpu().numpy()[0].reshape(4, cout).sum(0)
    close(s / (ref.size / cout), ref.reshape(-1, cout).mean(0), dt, "tconv stats")
    dout = rng.standard_normal((N, 2 * H, 2 * W, cout)).astype(np.float32)
    dx_ref, dk_ref, _ = R.tconv2x2s2_bwd(xr, kr, rnd(dout, dt))
    dx = torch.empty(N * H * W * cin, dtype=TDT[dt], device="cuda")
    ops.tconv_dgrad(d, dev(dout, dt), N, H, W, cout, kT, cin, dx)
    dk = torch.empty(2, 2, cout, cin, device="cuda")
    ops.tconv_wgrad(d, xv, dev(dout, dt), cout, dk)
    torch.cuda.synchronize()
    close(host(dx).reshape(dx_ref.shape), dx_ref, dt, "tconv dgrad")
    close(host(dk), dk_ref, dt, "tconv wgrad")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("cin,cout,H,W", [(512, 256, 5, 7), (256, 128, 9, 40)])
def test_tconv_affine_inference_epilogue(dt, cin, cout, H, W):
    """Conv2DTranspose forward with the inference BN affine after the ReLU (no sums): bf16 runs
    tconv_fwd2p_kernel, whose plan depends on the sizes only (the stat-row query matches
    whatever flags the launch carries)."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin + 1)
    N = 2
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    k = (rng.standard_normal((2, 2, cout, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    sc = rng.uniform(-2, 2, cout).astype(np.float32)
    sh = rng.standard_normal(cout).astype(np.float32)
    d = DT[dt]
    ref = np.maximum(R.tconv2x2s2(rnd(x, dt), rnd(k, dt), b), 0) * sc + sh
    kf = torch.empty(k.size, dtype=TDT[dt], device="cuda")
    kT = torch.empty(k.size, dtype=TDT[dt], device="cuda")
    ops.prep_tconv(d, torch.tensor(k).cuda(), cout, cin, kf, kT)
    out = torch.zeros(N * 2 * H * 2 * W * cout, dtype=TDT[dt], device="cuda")
    ops.tconv_fwd(d, ops.View(dev(x, dt).reshape(-1), N, H, W, cin, cin), kf, torch.tensor(b).cuda(),
                  ops.View(out, N, 2 * H, 2 * W, cout, cout, 0), flags=1 | 4,
                  aff=(torch.tensor(sc).cuda(), torch.tensor(sh).cuda()))
    torch.cuda.synchronize()
    close(host(out).reshape(ref.shape), ref, dt, "tconv affine")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_im2col_columns_exact(dt):
    """cnnitmo_im2col_c3 == the (r, s, c)-ordered 3x3x3 patches (+5 zero columns), bit-exact,
    over several 256-pixel row segments (the last one partial) and zero-padded rows >= Hv."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(10)
    N, Hv, H, W = 2, 5, 8, 300
    x = rng.uniform(size=(N, Hv, W, 3)).astype(np.float32)
    cols = torch.empty(N * H * W * 32, dtype=TDT[dt], device="cuda")
    ops.im2col_c3(DT[dt], torch.tensor(x).cuda(), N, Hv, H, W, cols)
    xp = np.zeros((N, H + 2, W + 2, 3), np.float32)
    xp[:, 1:Hv + 1, 1:W + 1] = x
    ref = np.zeros((N, H, W, 32), np.float32)
    for r in range(3):
        for c in range(3):
            ref[..., (r * 3 + c) * 3:(r * 3 + c) * 3 + 3] = xp[:, r:r + H, c:c + W]
    got = cols.float().cpu().numpy().reshape(N, H, W, 32)
    np.testing.assert_array_equal(got, rnd(ref, dt))


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_first_layer_im2col(dt):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(9)
    N, Hv, H, W = 2, 13, 16, 10
    x = rng.uniform(size=(N, Hv, W, 3)).astype(np.float32)
    w = (rng.standard_normal((32, 3, 3, 3)) * 0.3).astype(np.float32)
    b = rng.standard_normal(32).astype(np.float32)
    d = DT[dt]
    cols = torch.empty(N * H * W * 32, dtype=TDT[dt], device="cuda")
    ops.im2col_c3(d, torch.tensor(x).cuda(), N, Hv, H, W, cols)
    wp = torch.empty(32 * 32, dtype=TDT[dt], device="cuda")
    ops.prep_c3(d, torch.tensor(w).cuda(), 32, wp)
    out = ops.new_view(N, H, W, 32, TDT[dt])
    ops.conv1tap_fwd(d, cols, 32, N * H * W, wp, torch.tensor(b).cuda(), out, flags=1)
    xp = np.zeros((N, H, W, 3))
    xp[:, :Hv] = rnd(x, dt)
    ref = np.maximum(R.conv2d_same(xp, rnd(w, dt), b), 0)
    torch.cuda.synchronize()
    close(host(out.buf).reshape(ref.shape), ref, dt, "first layer")
    dz = rng.standard_normal((N, H, W, 32)).astype(np.float32)
    _, dw_ref, _ = R.conv2d_same_bwd(xp, rnd(w, dt), rnd(dz, dt), need_dx=False)
    dw = torch.empty(32, 27, device="cuda")
    ops.conv_wgrad(d, 1, ops.View(cols, N, H, W, 32, 32), dev(dz, dt), 32, dw, dw_cols=27)
    torch.cuda.synchronize()
    close(host(dw).reshape(dw_ref.shape), dw_ref, dt, "first layer wgrad")


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("N,Hv,H,W,ld,off", [(2, 13, 16, 10, 32, 0), (1, 6, 7, 300, 96, 64), (3, 9, 9, 256, 32, 0),
                                             (2, 5, 6, 517, 32, 0)])
def test_first_layer_direct(N, Hv, H, W, ld, off, dt):
    """cnnitmo_conv_c3_fwd (bf16 and fp32 outputs) / _wgrad (bf16), no im2col buffer, vs
    the oracle: ReLU + BN partial sums + output view, partial 256-pixel segments, zero
    rows >= Hv, odd widths (the edge piece of every row) and a row count that is not a
    multiple of the 4-row workgroup."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(19)
    x = rng.uniform(size=(N, Hv, W, 3)).astype(np.float32)
    w = (rng.standard_normal((32, 3, 3, 3)) * 0.3).astype(np.float32)
    b = rng.standard_normal(32).astype(np.float32)
    wp = torch.empty(32 * 32, dtype=TDT[dt], device="cuda")
    ops.prep_c3(DT[dt], torch.tensor(w).cuda(), 32, wp)
    buf = torch.zeros(N * H * W * ld, dtype=TDT[dt], device="cuda")
    out = ops.View(buf, N, H, W, 32, ld, off)
    rows = ops.conv_c3_stat_rows(N, H, W)
    stats = torch.empty(rows * 64, device="cuda")
    xd = torch.tensor(x).cuda()
    ops.conv_c3_fwd(DT[dt], xd, N, Hv, H, W, wp, torch.tensor(b).cuda(), out, flags=1 | 2, stats=stats)
    xp = np.zeros((N, H, W, 3))
    xp[:, :Hv] = rnd(x, dt)
    ref = np.maximum(R.conv2d_same(xp, rnd(w, dt), b), 0)
    torch.cuda.synchronize()
    got = host(buf).reshape(N, H, W, ld)[..., off:off + 32]
    close(got, ref, dt, "first layer direct")
    st = stats.cpu().numpy().reshape(rows, 2, 32).sum(0)
    np.testing.assert_allclose(st[0], ref.reshape(-1, 32).sum(0), rtol=2e-2, atol=2e-2 * ref.size / 32)
    np.testing.assert_allclose(st[1], (ref ** 2).reshape(-1, 32).sum(0), rtol=3e-2)
    dz = rng.standard_normal((N, H, W, 32)).astype(np.float32)
    _, dw_ref, _ = R.conv2d_same_bwd(xp, rnd(w, dt), rnd(dz, dt), need_dx=False)
    dw = torch.empty(32, 27, device="cuda")
    ops.conv_c3_wgrad(DT[dt], xd, N, Hv, H, W, dev(dz, dt), dw)
    torch.cuda.synchronize()
    close(host(dw).reshape(dw_ref.shape), dw_ref, dt, "first layer direct wgrad")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_maxpool_ties(dt):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(4)
    N, H, W, C, ld, off = 2, 6, 8, 32, 96, 64
    xb = rng.integers(-2, 3, size=(N, H, W, ld)).astype(np.float32)  # many ties
    d = DT[dt]
    xv = ops.View(dev(xb, dt).reshape(-1), N, H, W, C, ld, off)
    y = torch.empty(N * H // 2 * W // 2 * C, dtype=TDT[dt], device="cuda")
    idx = torch.empty(N * H // 2 * W // 2 * C, dtype=torch.uint8, device="cuda")
    ops.maxpool_fwd(d, xv, y, idx)
    yr, ir = R.maxpool2x2(xb[..., off:].astype(np.float64))
    dy = rng.standard_normal(yr.shape).astype(np.float32)
    base = rng.standard_normal((N, H, W, ld)).astype(np.float32)
    dxb = dev(base, dt).reshape(-1)
    ops.maxpool_bwd(d, dev(dy, dt), idx, ops.View(dxb, N, H, W, C, ld, off))
    torch.cuda.synchronize()
    assert np.array_equal(host(y).reshape(yr.shape), yr)
    assert np.array_equal(idx.cpu().numpy().reshape(ir.shape), ir)
    want = rnd(base, dt)
    want[..., off:] += R.maxpool2x2_bwd(rnd(dy, dt), ir, (N, H, W, C))
    close(host(dxb).reshape(want.shape), want, dt, "pool bwd")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("drop", [False, True])
@pytest.mark.parametrize("C", [64, 96])  # (96: bn_apply's generic, non-power-of-two index path)
def test_bn_train_fwd_bwd(dt, drop, C):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(5)
    N, H, W = 2, 5, 7
    P = N * H * W
    r = np.maximum(rng.standard_normal((N, H, W, C)), 0).astype(np.float32)
    g = rng.uniform(0.5, 1.5, C).astype(np.float32)
    be = rng.standard_normal(C).astype(np.float32)
    rr = rnd(r, dt)
    d = DT[dt]
    rt = dev(r, dt)
    # stats as the conv epilogue would produce them (one row)
    stats = torch.tensor(np.stack([rr.reshape(-1, C).sum(0), (rr.reshape(-1, C) ** 2).sum(0)])[None],
                         dtype=torch.float32).cuda()
    cu = lambda a: torch.tensor(a, dtype=torch.float32).cuda()
    mm, mv = cu(np.zeros(C)), cu(np.ones(C))
    sc, sh, sm, si = (torch.empty(C, device="cuda") for _ in range(4))
    ops.bn_fwd_finalize(stats, 1, C, 1, P, cu(g), cu(be), mm, mv, 0.99, 1e-3, sc, sh, sm, si)
    ld, off = C + 32, 32
    yb = torch.zeros(P * ld, dtype=TDT[dt], device="cuda")
    seed, layer = 123, 1
    ops.bn_apply(d, rt, P, C, sc, sh, ops.View(yb, N, H, W, C, ld, off), flags=1 if drop else 0,
                 seed=seed, layer=layer)
    y_ref, m_ref, v_ref = R.bn_train_fwd(rr, g, be)
    if drop:
        y_ref, keep = R.dropout_fwd(y_ref, seed, layer)
    mm_ref, mv_ref = R.bn_moving_update(np.zeros(C), np.ones(C), m_ref, v_ref, P)
    torch.cuda.synchronize()
    close(host(yb).reshape(N, H, W, ld)[..., off:], y_ref, dt, "bn apply")
    np.testing.assert_allclose(mm.cpu().numpy(), mm_ref, atol=1e-5)
    np.testing.assert_allclose(mv.cpu().numpy(), mv_ref, atol=1e-5)
    # backward from a dy view
    dyb = rng.standard_normal((N, H, W, ld)).astype(np.float32)
    dy = rnd(dyb, dt)[..., off:]
    dyv = ops.View(dev(dyb, dt).reshape(-1), N, H, W, C, ld, off)
    flags = 1 if drop else 0
    rows = ops.bn_bwd_rows(P, C)
    part = torch.empty(rows, 2, C, device="cuda")
    ops.bn_bwd_reduce(d, dyv, rt, C, sm, si, flags, seed, layer, part)
    dgam, dbet, coef = torch.empty(C, device="cuda"), torch.empty(C, device="cuda"), torch.empty(3, C, device="cuda")
    ops.bn_bwd_finalize(part, rows, C, P, cu(g), sm, si, dgam, dbet, coef)
    dz = torch.empty(P * C, dtype=TDT[dt], device="cuda")
    part2 = torch.empty(rows, C, device="cuda")
    ops.bn_bwd_apply(d, dyv, rt, C, coef, flags, seed, layer, dz, part2)
    db = torch.empty(C, device="cuda")
    ops.colsum(part2, rows, C, 1, db)
    dyd = dy * keep * 2.0 if drop else dy
    dr, dg_ref, dbeta_ref = R.bn_train_bwd(dyd, rr, g, m_ref, v_ref)
    dz_ref = dr * (rr > 0)
    torch.cuda.synchronize()
    close(host(dgam), dg_ref, dt, "dgamma")
    close(host(dbet), dbeta_ref, dt, "dbeta")
    close(host(dz).reshape(dz_ref.shape), dz_ref, dt, "dz")
    close(host(db), dz_ref.reshape(-1, C).sum(0), dt, "db")


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("C,H,W", [(64, 8, 16),
                                   # head2_kernel at 2..16 lanes per pixel, ragged 64-pixel groups
                                   (16, 5, 13), (32, 9, 31), (128, 6, 11),
                                   # head_kernel (32 / 64 lanes per pixel)
                                   (256, 4, 9)])
def test_head(dt, C, H, W):
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(6 + C)
    N, Hv = 2, H - 1
    x = rng.standard_normal((N, H, W, C)).astype(np.float32)
    w = (rng.standard_normal((3, C)) * 0.2).astype(np.float32)
    b = rng.standard_normal(3).astype(np.float32)
    t = rng.uniform(size=(N, Hv, W, 3)).astype(np.float32)
    d = DT[dt]
    xv = ops.View(dev(x, dt).reshape(-1), N, H, W, C, C)
    cu = lambda a: torch.tensor(a, dtype=torch.float32).cuda()
    yh = torch.empty(N, Hv, W, 3, device="cuda")
    ops.head_fwd(d, xv, Hv, cu(w), cu(b), yh)
    xr = rnd(x, dt)[:, :Hv]
    yref = R.sigmoid(xr @ w.T.astype(np.float64) + b)
    rows = ops.head_rows(N * H * W)
    part = torch.empty(rows, 5 + 3 * C, device="cuda")
    dx = torch.empty(N * H * W * C, dtype=TDT[dt], device="cuda")
    ops.head_fwd_bwd(d, xv, Hv, cu(w), cu(b), cu(t), dx, part)
    la, dw, db = torch.empty(2, device="cuda"), torch.empty(3, C, device="cuda"), torch.empty(3, device="cuda")
    ops.head_finalize(part, rows, C, N * Hv * W * 3, la, dw, db)
    dz = R.mse_grad_z(yref, t)
    dx_ref = np.zeros((N, H, W, C))
    dx_ref[:, :Hv] = dz @ w.astype(np.float64)
    torch.cuda.synchronize()
    close(yh.cpu().numpy(), yref, "f32", "yhat")
    assert abs(la[0].item() - R.mse(yref, t)) < 1e-5
    assert abs(la[1].item() - R.categorical_accuracy(t, yref)) < 1e-6
    close(host(dw), dz.reshape(-1, 3).T @ xr.reshape(-1, C), "f32", "head dw")
    close(host(db), dz.reshape(-1, 3).sum(0), "f32", "head db")
    close(host(dx).reshape(dx_ref.shape) * 1e3, dx_ref * 1e3, dt, "head dx")
    # the rank-3 gradient form: g3 = dz per pixel (zeros on the padding rows), same sums
    g3 = torch.full((N * H * W * 3,), 7.0, device="cuda")
    part3 = torch.empty(rows, 5 + 3 * C, device="cuda")
    ops.head_fwd_bwd_g3(d, xv, Hv, cu(w), cu(b), cu(t), g3, part3)
    la3, dw3, db3 = torch.empty(2, device="cuda"), torch.empty(3, C, device="cuda"), torch.empty(3, device="cuda")
    ops.head_finalize(part3, rows, C, N * Hv * W * 3, la3, dw3, db3)
    g3_ref = np.zeros((N, H, W, 3))
    g3_ref[:, :Hv] = dz
    torch.cuda.synchronize()
    close(g3.cpu().numpy().reshape(g3_ref.shape) * 1e3, g3_ref * 1e3, "f32", "head g3")
    assert np.array_equal(la3.cpu().numpy(), la.cpu().numpy())
    assert np.array_equal(host(dw3), host(dw)) and np.array_equal(host(db3), host(db))


def test_rmsprop():
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(7)
    n = 1003
    p, g, a = rng.standard_normal(n), rng.standard_normal(n), rng.uniform(size=n)
    pt, gt, at = (torch.tensor(v, dtype=torch.float32).cuda() for v in (p, g, a))
    ops.rmsprop(pt, gt, at, 1e-3, 0.9, 1e-7, grad_scale=0.5)
    pr, ar = R.rmsprop(p, g * 0.5, a)
    torch.cuda.synchronize()
    np.testing.assert_allclose(pt.cpu().numpy(), pr, atol=1e-6)
    np.testing.assert_allclose(at.cpu().numpy(), ar, atol=1e-6)


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("cin,cout,H,W", [(32, 32, 16, 64), (64, 64, 18, 70), (128, 128, 8, 96), (64, 64, 6, 34)])
def test_conv3x3_fwd_pool(dt, cin, cout, H, W):
    """cnnitmo_conv3x3_fwd_pool: the conv output is the plain conv3x3_fwd's bit for bit,
    and the pooled value / window index are the first-max rule applied to the STORED
    output with the per-channel mode sign(pool_sign) (max, min, first) -- and plain max
    without a sign (inference).  Partial tiles in both directions (W % 32, H % 16)."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(cin + H)
    N = 2
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.1).astype(np.float32)
    b = rng.standard_normal(cout).astype(np.float32)
    d, T = DT[dt], TDT[dt]
    if not ops.pool_supported(d, N, H, W, cin, cout):
        pytest.skip("halo kernel does not take this shape")
    wf = torch.empty(w.size, dtype=T, device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cin, wf, None)
    xv = ops.View(dev(x, dt).reshape(-1), N, H, W, cin, cin)
    bias = torch.tensor(b).cuda()
    ref = ops.new_view(N, H, W, cout, T)
    rows = ops.conv3x3_stat_rows(d, N, H, W, cin, cout)
    st0 = torch.zeros(rows * 2 * cout, device="cuda")
    ops.conv3x3_fwd(d, xv, wf, bias, ref, 1 | 2, stats=st0)
    sign = torch.tensor(np.resize([1.0, -0.5, 0.0, 3.0], cout).astype(np.float32)).cuda()
    for sg in (sign, None):
        out = ops.new_view(N, H, W, cout, T)
        pv = torch.empty(N * (H // 2) * (W // 2) * cout, dtype=T, device="cuda")
        pi = torch.empty(N * (H // 2) * (W // 2) * cout, dtype=torch.uint8, device="cuda")
        st = torch.zeros(rows * 2 * cout, device="cuda")
        ops.conv3x3_fwd_pool(d, xv, wf, bias, out, pv, pi, sg, flags=1 | 2, stats=st)
        torch.cuda.synchronize()
        assert torch.equal(out.buf, ref.buf)
        assert torch.allclose(st.view(rows, 2, cout).sum(0), st0.view(rows, 2, cout).sum(0), rtol=1e-5, atol=1e-3)
        y = ref.buf.view(N, H // 2, 2, W // 2, 2, cout).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, cout)
        m = torch.ones(cout, device="cuda") if sg is None else torch.sign(sg)
        key = y.double() * m.double()
        first = (key == key.max(3, keepdim=True).values).to(torch.uint8).argmax(3)
        assert torch.equal(pi.view(N, H // 2, W // 2, cout), first.to(torch.uint8))
        assert torch.equal(pv.view(N, H // 2, W // 2, cout), y.gather(3, first.unsqueeze(3)).squeeze(3))
    # the inference kernel predict() launches: ReLU + the BN affine (negative scales too) applied
    # before pooling, no sums (the NOSUM instantiation); pooled by the maximum of the stored y
    sc = torch.tensor(np.resize([1.5, -0.75, 0.25, -2.0], cout).astype(np.float32)).cuda()
    sh = torch.tensor(rng.standard_normal(cout).astype(np.float32)).cuda()
    refa = ops.new_view(N, H, W, cout, T)
    ops.conv3x3_fwd(d, xv, wf, bias, refa, 1 | 4, aff=(sc, sh))
    out = ops.new_view(N, H, W, cout, T)
    pv = torch.empty(N * (H // 2) * (W // 2) * cout, dtype=T, device="cuda")
    pi = torch.empty(N * (H // 2) * (W // 2) * cout, dtype=torch.uint8, device="cuda")
    ops.conv3x3_fwd_pool(d, xv, wf, bias, out, pv, pi, None, flags=1 | 4, aff=(sc, sh))
    torch.cuda.synchronize()
    assert torch.equal(out.buf, refa.buf)
    y = refa.buf.view(N, H // 2, 2, W // 2, 2, cout).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, cout)
    key = y.double()
    first = (key == key.max(3, keepdim=True).values).to(torch.uint8).argmax(3)
    assert torch.equal(pi.view(N, H // 2, W // 2, cout), first.to(torch.uint8))
    assert torch.equal(pv.view(N, H // 2, W // 2, cout), y.gather(3, first.unsqueeze(3)).squeeze(3))


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("cin,H,W,hv", [(64, 18, 70, 17), (96, 16, 64, 16), (64, 5, 33, 3)])
def test_conv3x3_fwd_head(dt, cin, H, W, hv):
    """cnnitmo_conv3x3_fwd_head (model.py:262-264 in predict): conv3x3 + ReLU + the inference
    BN affine + the 1x1 sigmoid head, the conv output never stored, vs the fp64 oracle on
    operands rounded to dtype (the conv accumulates in fp32 and is not rounded to dtype).
    Partial tiles, valid rows < h."""
    from cnn_itmo_amd import ops
    from cnn_itmo_amd import _lib as L
    rng = np.random.default_rng(cin + H + hv)
    N, cout = 2, 64
    x = rng.standard_normal((N, H, W, cin)).astype(np.float32)
    w = (rng.standard_normal((cout, 3, 3, cin)) * 0.05).astype(np.float32)
    b = (rng.standard_normal(cout) * 0.1).astype(np.float32)
    s, h = rng.uniform(0.5, 1.5, cout).astype(np.float32), rng.normal(0, 0.2, cout).astype(np.float32)
    hw = (rng.standard_normal((3, cout)) * 0.2).astype(np.float32)
    hb = rng.standard_normal(3).astype(np.float32)
    d, T = DT[dt], TDT[dt]
    if not ops.head_supported(d, N, H, W, cin, cout):
        pytest.skip("halo kernel does not take this shape")
    wf = torch.empty(w.size, dtype=T, device="cuda")
    ops.prep_conv3x3(d, torch.tensor(w).cuda(), cout, cin, wf, None)
    xv = ops.View(dev(x, dt).reshape(-1), N, H, W, cin, cin)
    yhat = torch.full((N, hv, W, 3), -1.0, device="cuda")
    ops.conv3x3_fwd_head(d, xv, wf, torch.tensor(b).cuda(), cout, L.RELU | L.AFFINE,
                         (torch.tensor(s).cuda(), torch.tensor(h).cuda()), hv, torch.tensor(hw).cuda(),
                         torch.tensor(hb).cuda(), yhat)
    torch.cuda.synchronize()
    y = np.maximum(R.conv2d_same(rnd(x, dt), rnd(w, dt), b), 0) * s + h
    z = y[:, :hv] @ hw.T.astype(np.float64) + hb
    ref = 1.0 / (1.0 + np.exp(-z))
    np.testing.assert_allclose(host(yhat), ref, rtol=0, atol=2e-5 if dt == "f32" else 5e-5)


@pytest.mark.parametrize("H,W", [(16, 64), (20, 70), (8, 40)])
def test_conv3x3_fwd_cat_dec9(H, W):
    """cnnitmo_conv3x3_fwd_cat on dec9's shape ([conv1 32 | up9 64] -> 64, model.py:261-262)
    vs the oracle on the materialised concat: ReLU + BN sums (16-row tiles, the two
    members read per 32-channel chunk)."""
    from cnn_itmo_amd import ops
    rng = np.random.default_rng(H + W)
    N = 2
    x1 = rng.standard_normal((N, H, W, 32)).astype(np.float32)
    x2 = rng.standard_normal((N, H, W, 64)).astype(np.float32)
    w = (rng.standard_normal((64, 3, 3, 96)) * 0.1).astype(np.float32)
    b = rng.standard_normal(64).astype(np.float32)
    wf = torch.empty(w.size, dtype=torch.bfloat16, device="cuda")
    ops.prep_conv3x3(1, torch.tensor(w).cuda(), 64, 96, wf, None)
    v1 = ops.View(dev(x1, "bf16").reshape(-1), N, H, W, 32, 32)
    v2 = ops.View(dev(x2, "bf16").reshape(-1), N, H, W, 64, 64)
    out = ops.new_view(N, H, W, 64, torch.bfloat16)
    rows = ops.conv3x3_stat_rows(1, N, H, W, 96, 64)
    st = torch.zeros(rows * 128, device="cuda")
    ops.conv3x3_fwd_cat(1, v1, v2, wf, torch.tensor(b).cuda(), out, 1 | 2, stats=st)
    torch.cuda.synchronize()
    xc = np.concatenate([rnd(x1, "bf16"), rnd(x2, "bf16")], 3).astype(np.float64)
    ref = np.maximum(R.conv2d_same(xc, rnd(w, "bf16").astype(np.float64), b), 0)
    got = host(out.buf).reshape(ref.shape)
    err = float(np.abs(got - ref).max()) / max(1.0, float(np.abs(ref).max()))
    s = st.view(rows, 2, 64).double().sum(0).cpu().numpy()
    serr = float(np.abs(s[0] - got.reshape(-1, 64).sum(0)).max()) / max(1.0, float(np.abs(got).sum()))
    assert err <= 1.5e-2 and serr <= 1e-5, (err, serr)
