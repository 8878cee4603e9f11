"""CPU checks of the per-launch checker itself (tests/launch_check*.py).

The full-size GPU parity tests (test_gpu_benchshapes.py) are only as good as the
checks they run.  Here every non-GEMM check is fed (a) outputs produced by an fp32
emulation of the kernel's contract -- it must accept them -- and (b) the same
outputs with one element perturbed -- it must reject them.  The Dropout hash of
the checker (torch int64) is pinned to the oracle's (numpy uint64).
"""
import types

import numpy as np
import pytest
import torch

from cnn_itmo_amd import _lib as L
from cnn_itmo_amd.ops import View
from launch_check import LAUNCHES, LaunchChecker
from launch_check_elem import dropout_keep
from oracle import unet_ref as R

F32, BF = torch.float32, torch.bfloat16


def _checker(dt):
    ops = types.SimpleNamespace(**{k: (lambda *a, **kw: None) for k in LAUNCHES})
    ops.call = lambda *a: 0
    return LaunchChecker(ops, dt, verbose=False)


def _fails(fn, *a, **k):
    with pytest.raises(AssertionError):
        fn(*a, **k)


def _bump(t, i=3, by=None):
    t = t.clone()
    f = t.view(-1)
    v = float(f[i])
    f[i] = v + (by if by is not None else 0.25 * abs(v) + 1e-3)
    return t


def test_dropout_hash_matches_oracle():
    for seed, layer in [(0, 1), (3, 2), (123456789, 1), (2 ** 40 + 7, 2)]:
        for start in (0, 2 ** 33 - 5):
            idx = torch.arange(start, start + 4096, dtype=torch.int64)
            got = dropout_keep(seed, layer, idx).numpy()
            ref = R.dropout_keep(seed, layer, 4096, start)
            assert (got == ref).all()
            assert 0.4 < got.mean() < 0.6


@pytest.mark.parametrize("dt", [L.BF16, L.F32])
def test_maxpool_checks(dt):
    T = BF if dt == L.BF16 else F32
    g = torch.Generator().manual_seed(0)
    n, h, w, c = 2, 6, 8, 16
    x = (torch.randint(0, 5, (n * h * w * c,), generator=g).float() / 4).to(T)  # many exact ties
    xv = View(x, n, h, w, c, c)
    chk = _checker(dt)
    # raw input (bit-exact path), emulated by the oracle's first-max pool
    y, idx = R.maxpool2x2(x.float().numpy().reshape(n, h, w, c))
    yt, it = torch.from_numpy(y).to(T).reshape(-1), torch.from_numpy(idx).reshape(-1)
    chk._chk_maxpool_fwd(dt, xv, yt, it)
    bad = it.clone()
    k = int(((it == 0).nonzero())[0])  # a window whose first max is element 0 ...
    bad[k] = 3
    _fails(chk._chk_maxpool_fwd, dt, xv, yt, bad)
    # folded BN input: the pool sees r*s + h in fp32 (negative scales flip the order)
    s = torch.randn(c, generator=g)
    sh = torch.randn(c, generator=g)
    v = (x.float().view(n, h, w, c) * s + sh)
    y2, idx2 = R.maxpool2x2(v.numpy())
    y2t, i2t = torch.from_numpy(y2).to(T).reshape(-1), torch.from_numpy(idx2).reshape(-1)
    chk._chk_maxpool_fwd(dt, xv, y2t, i2t, aff=(s, sh))
    _fails(chk._chk_maxpool_fwd, dt, xv, _bump(y2t.float()).to(T), i2t, aff=(s, sh))
    # backward: scatter-add into an existing gradient slice of a wider buffer
    ld = c + 8
    buf = torch.randn(n * h * w * ld, generator=g).to(T)
    dxv = View(buf, n, h, w, c, ld, 8)
    pre = dxv.tensor().clone()
    dy = torch.randn(n * (h // 2) * (w // 2) * c, generator=g).to(T)
    add = R.maxpool2x2_bwd(dy.float().numpy().reshape(n, h // 2, w // 2, c), idx, (n, h, w, c))
    hit = R.maxpool2x2_bwd(np.ones((n, h // 2, w // 2, c), np.float32), idx, (n, h, w, c)) > 0
    new = torch.where(torch.from_numpy(hit), (pre.float() + torch.from_numpy(add)).to(T), pre)
    dxv.tensor().copy_(new)
    chk._chk_maxpool_bwd(dt, dy, it, dxv, pre=pre)
    dxv.tensor()[0, 0, 0, 0] += 1.0
    _fails(chk._chk_maxpool_bwd, dt, dy, it, dxv, pre=pre)


def _bn_setup(dt, n=2, h=6, w=8, c=16, seed=1):
    T = BF if dt == L.BF16 else F32
    g = torch.Generator().manual_seed(seed)
    r = torch.relu(torch.randn(n * h * w * c, generator=g)).to(T)
    return g, T, r, View(r, n, h, w, c, c)


def test_bn_forward_checks():
    dt = L.BF16
    g, T, r, rv = _bn_setup(dt)
    c, p = rv.c, rv.p
    chk = _checker(dt)
    rows = 5  # partial rows as the conv epilogue writes them: [rows][2][c]
    rf = r.float().view(p, c)
    st = torch.zeros(rows, 2, c)
    for k in range(rows):
        blk = rf[k::rows]
        st[k, 0], st[k, 1] = blk.sum(0), (blk * blk).sum(0)
    gamma, beta = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g)
    mm0, mv0 = torch.randn(c, generator=g), torch.rand(c, generator=g) + 0.5
    mean = st[:, 0].double().sum(0) / p
    var = st[:, 1].double().sum(0) / p - mean * mean
    inv = 1 / torch.sqrt(var + 1e-3)
    sc = gamma.double() * inv
    mmn, mvn = R.bn_moving_update(mm0.double().numpy(), mv0.double().numpy(), mean.numpy(), var.numpy(), p,
                                  momentum=float(np.float32(0.99)), eps=float(np.float32(1e-3)))
    outs = [sc.float(), (beta.double() - mean * sc).float(), mean.float(), inv.float()]
    mm, mv = torch.from_numpy(mmn).float(), torch.from_numpy(mvn).float()
    args = (st.view(-1), rows, c, 1, p, gamma, beta, mm, mv, 0.99, 1e-3)
    chk._chk_bn_fwd_finalize(*args, *outs, pre=(mm0, mv0))
    _fails(chk._chk_bn_fwd_finalize, *args, *outs, pre=(mm0, mv0 * 1.01))  # wrong moving-variance input
    _fails(chk._chk_bn_fwd_finalize, *args, outs[0], _bump(outs[1]), *outs[2:], pre=(mm0, mv0))
    # inference coefficients
    s2 = (gamma / torch.sqrt(mv + np.float32(1e-3)))
    chk._chk_bn_infer_coeffs(c, gamma, beta, mm, mv, 1e-3, s2, beta - mm * s2)
    _fails(chk._chk_bn_infer_coeffs, c, gamma, beta, mm, mv, 1e-3, _bump(s2), beta - mm * s2)
    # BN apply + Dropout(0.5) into a concat slice
    ld = c + 16
    y = torch.zeros(p * ld).to(T)
    yv = View(y, rv.n, rv.h, rv.w, c, ld, 16)
    keep = torch.from_numpy(R.dropout_keep(7, 2, p * c)).view(p, c)
    out = torch.where(keep, 2 * (rf * outs[0] + outs[1]), torch.zeros(()))
    yv.tensor().copy_(out.view(rv.n, rv.h, rv.w, c).to(T))
    chk._chk_bn_apply(dt, r, p, c, outs[0], outs[1], yv, L.DROPOUT, 7, 2)
    _fails(chk._chk_bn_apply, dt, r, p, c, outs[0], outs[1], yv, L.DROPOUT, 8, 2)  # another seed's mask


@pytest.mark.parametrize("flags", [0, L.DROPOUT, L.PARITY, L.NO_BN])
def test_bn_backward_checks(flags):
    dt = L.BF16
    g, T, r, rv = _bn_setup(dt)
    n, h, w, c, p = rv.n, rv.h, rv.w, rv.c, rv.p
    chk = _checker(dt)
    dy = torch.randn(p * c, generator=g).to(T)
    dyv = View(dy, n, h, w, c, c)
    d = dy.float().view(p, c)
    if flags & L.DROPOUT:
        keep = torch.from_numpy(R.dropout_keep(5, 1, p * c)).view(p, c)
        d = torch.where(keep, 2 * d, torch.zeros(()))
    mean, inv = torch.rand(c, generator=g), torch.rand(c, generator=g) + 0.5
    rf = r.float().view(p, c)
    rows = 3
    part = torch.zeros(rows, 2, c)
    for k in range(rows):
        part[k, 0] = d[k::rows].sum(0)
        part[k, 1] = (d[k::rows] * (rf[k::rows] - mean) * inv).sum(0)
    if not flags & (L.PARITY | L.NO_BN):
        chk._chk_bn_bwd_reduce(dt, dyv, r, c, mean, inv, flags, 5, 1, part.view(-1))
        _fails(chk._chk_bn_bwd_reduce, dt, dyv, r, c, mean, inv, flags, 5, 1, _bump(part.view(-1)))
    gamma = torch.rand(c, generator=g) + 0.5
    sdy, sdyr = part[:, 0].double().sum(0), part[:, 1].double().sum(0)
    a = gamma.double() * inv
    b = a * inv * sdyr / p
    e = b * mean - a * sdy / p
    coef = torch.cat([a, b, e]).float()
    chk._chk_bn_bwd_finalize(part.view(-1), rows, c, p, gamma, mean, inv, sdyr.float(), sdy.float(), coef)
    _fails(chk._chk_bn_bwd_finalize, part.view(-1), rows, c, p, gamma, mean, inv, sdyr.float(), sdy.float(),
           _bump(coef, 2 * c + 1))
    ca, cb, ce = coef.view(3, c)
    dz = torch.where(rf > 0, d if flags & L.NO_BN else ca * d - cb * rf + ce, torch.zeros(())).to(T)
    npar = 4 if flags & L.PARITY else 1
    zs = dz.float().view(n, h, w, c)
    pp = torch.zeros(2, npar, c)
    for k in range(npar):
        v = zs[:, k >> 1::2, k & 1::2] if npar == 4 else zs
        pp[0, k] = v.reshape(-1, c)[0::2].sum(0)
        pp[1, k] = v.reshape(-1, c)[1::2].sum(0)
    cf = None if flags & L.NO_BN else coef
    chk._chk_bn_bwd_apply(dt, dyv, r, c, cf, flags, 5, 1, dz.view(-1), pp.view(-1))
    _fails(chk._chk_bn_bwd_apply, dt, dyv, r, c, cf, flags, 5, 1, _bump(dz.float().view(-1), 9).to(T), pp.view(-1))
    _fails(chk._chk_bn_bwd_apply, dt, dyv, r, c, cf, flags, 5, 1, dz.view(-1), _bump(pp.view(-1), 1))


def test_bn_backward_routed_and_g3():
    dt = L.BF16
    g, T, r, rv = _bn_setup(dt)
    n, h, w, c, p = rv.n, rv.h, rv.w, rv.c, rv.p
    chk = _checker(dt)
    coef = torch.cat([torch.rand(c, generator=g) + .5, torch.rand(c, generator=g), torch.randn(c, generator=g)])
    ca, cb, ce = coef.view(3, c)
    rf = r.float().view(p, c)
    # pooled route: dy + the pool gradient routed by argmax
    dy = torch.randn(p * c, generator=g).to(T)
    dyp = torch.randn(p // 4 * c, generator=g).to(T)
    idx = torch.randint(0, 4, (p // 4 * c,), generator=g, dtype=torch.uint8)
    add = R.maxpool2x2_bwd(dyp.float().numpy().reshape(n, h // 2, w // 2, c), idx.numpy().reshape(n, h // 2, w // 2, c),
                           (n, h, w, c))
    gg = dy.float().view(p, c) + torch.from_numpy(add).view(p, c)
    dz = torch.where(rf > 0, ca * gg - cb * rf + ce, torch.zeros(())).to(T)
    part = dz.float().sum(0)
    dyv = View(dy, n, h, w, c, c)
    chk._chk_bn_bwd_apply_pooled(dt, dyv, rv, c, coef, dyp, idx, dz.view(-1), part)
    bad = idx.clone()
    bad[0] = (int(bad[0]) + 1) % 4
    _fails(chk._chk_bn_bwd_apply_pooled, dt, dyv, rv, c, coef, dyp, bad, dz.view(-1), part)
    # rank-3 head gradient
    g3 = torch.randn(p * 3, generator=g)
    wh = torch.randn(3 * c, generator=g)
    gg = g3.view(p, 3) @ wh.view(3, c)
    dz = torch.where(rf > 0, ca * gg - cb * rf + ce, torch.zeros(())).to(T)
    chk._chk_bn_bwd_apply_g3(dt, g3, wh, rv, c, p, coef, dz.view(-1), dz.float().sum(0))
    _fails(chk._chk_bn_bwd_apply_g3, dt, g3, _bump(wh), rv, c, p, coef, dz.view(-1), dz.float().sum(0))
    # the pool's share of the BN sums
    mean, inv = torch.rand(c, generator=g), torch.rand(c, generator=g) + 0.5
    win = rf.view(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(-1, 4, c)
    rsel = win.gather(1, idx.long().view(-1, 1, c)).squeeze(1)
    gp = dyp.float().view(-1, c)
    ps = torch.stack([gp.sum(0), (gp * (rsel - mean) * inv).sum(0)])
    chk._chk_pool_bnsums(dt, dyp, idx, rv, mean, inv, ps.view(-1))
    _fails(chk._chk_pool_bnsums, dt, dyp, idx, rv, mean, inv, _bump(ps.view(-1), c + 2))


def test_head_checks():
    dt = L.BF16
    g = torch.Generator().manual_seed(3)
    n, h, hv, w, cin = 2, 6, 5, 8, 64
    x = torch.relu(torch.randn(n * h * w * cin, generator=g)).to(BF)
    xv = View(x, n, h, w, cin, cin)
    wt, b = torch.randn(3 * cin, generator=g) * 0.1, torch.randn(3, generator=g) * 0.1
    s, sh = torch.rand(cin, generator=g) + 0.5, torch.randn(cin, generator=g) * 0.1
    t = (torch.randint(0, 256, (n * hv * w * 3,), generator=g).float() / 255)
    chk = _checker(dt)
    xi = x.float().view(n, h, w, cin)
    z = (xi * s + sh) @ wt.view(3, cin).t() + b
    y = torch.sigmoid(z)
    numel = n * hv * w * 3
    e = y[:, :hv] - t.view(n, hv, w, 3)
    d = torch.zeros(n, h, w, 3)
    d[:, :hv] = 2 * e * y[:, :hv] * (1 - y[:, :hv]) * np.float32(1.0 / numel)
    corr = float((t.view(n, hv, w, 3).argmax(-1) == y[:, :hv].argmax(-1)).sum())
    part = torch.cat([torch.tensor([float((e * e).sum()), corr]), d.view(-1, 3).sum(0),
                      (d.view(-1, 3).t() @ xi.view(-1, cin)).view(-1)])[None]
    chk._chk_head_fwd_bwd_g3(dt, xv, hv, wt, b, t, d.view(-1), part.view(-1), aff=(s, sh))
    _fails(chk._chk_head_fwd_bwd_g3, dt, xv, hv, wt, b, t, _bump(d.view(-1), 7), part.view(-1), aff=(s, sh))
    bad = part.clone()
    bad[0, 1] += 1
    _fails(chk._chk_head_fwd_bwd_g3, dt, xv, hv, wt, b, t, d.view(-1), bad.view(-1), aff=(s, sh))
    # finalize
    pr = torch.cat([part, torch.zeros_like(part)])
    tot = part[0].double()
    la = torch.tensor([tot[0] / numel, tot[1] / (numel / 3)]).float()
    dw = (tot[5:].view(3, cin) * s.double() + tot[2:5, None] * sh.double()).float().view(-1)
    chk._chk_head_finalize(pr.view(-1), 2, cin, numel, la, dw, tot[2:5].float(), aff=(s, sh),
                           raw=tot[5:].float())
    _fails(chk._chk_head_finalize, pr.view(-1), 2, cin, numel, la, dw, tot[2:5].float(), aff=None)
    # inference forward (no fold)
    yi = torch.sigmoid(xi @ wt.view(3, cin).t() + b)[:, :hv].reshape(-1)
    chk._chk_head_fwd(dt, xv, hv, wt, b, yi)
    _fails(chk._chk_head_fwd, dt, xv, hv, wt, b, _bump(yi, by=1e-4))


def test_rmsprop_prep_fold_reduce_checks():
    g = torch.Generator().manual_seed(4)
    n = 1000
    p0, g0, a0 = torch.randn(n, generator=g), torch.randn(n, generator=g) * 1e-2, torch.rand(n, generator=g) * 1e-4
    chk = _checker(L.BF16)
    gs = np.float32(0.5)
    gr = g0 * gs
    a1 = np.float32(0.9) * a0 + (np.float32(1) - np.float32(0.9)) * gr * gr
    p1 = p0 - np.float32(1e-3) * gr / (torch.sqrt(a1) + np.float32(1e-7))
    chk._chk_rmsprop(p1, g0, a1, 1e-3, 0.9, 1e-7, 0.5, pre=(p0, a0))
    _fails(chk._chk_rmsprop, p1, g0, a1, 1e-3, 0.9, 1e-7, 1.0, pre=(p0, a0))  # unscaled gradient
    # weight preparation (bit-exact) and BN folding
    cout, cin = 8, 16
    W = torch.randn(cout * 9 * cin, generator=g)
    wf = W.to(BF)
    wflip = W.view(cout, 3, 3, cin).flip(1, 2).permute(3, 1, 2, 0).contiguous().to(BF).view(-1)
    chk._chk_prep_conv3x3(L.BF16, W, cout, cin, wf, wflip)
    _fails(chk._chk_prep_conv3x3, L.BF16, W, cout, cin, wf, W.view(cout, 3, 3, cin).permute(3, 1, 2, 0).contiguous()
           .to(BF).view(-1))  # not flipped
    K = torch.randn(4 * cout * cin, generator=g)
    chk._chk_prep_tconv(L.BF16, K, cout, cin, K.to(BF), K.view(4, cout, cin).permute(2, 0, 1).contiguous().to(BF))
    w27 = torch.randn(cout * 27, generator=g)
    wp = torch.zeros(cout, 32)
    wp[:, :27] = w27.view(cout, 27)
    chk._chk_prep_c3(L.BF16, w27, cout, wp.to(BF))
    s, sh, bias = torch.rand(cin, generator=g) + .5, torch.randn(cin, generator=g), torch.randn(cout, generator=g)
    u = W.view(cout, 9, cin).double() @ sh.double()
    bo = (bias.double() + u.sum(1)).float()
    U = torch.stack([u[:, 0] + u[:, 1] + u[:, 2], u[:, 6] + u[:, 7] + u[:, 8], u[:, 0] + u[:, 3] + u[:, 6],
                     u[:, 2] + u[:, 5] + u[:, 8], u[:, 0], u[:, 2], u[:, 6], u[:, 8]], 1).float().view(-1)
    wo = (W.view(cout, 9, cin) * s).to(BF).view(-1)
    chk._chk_fold_conv3x3(L.BF16, W, bias, s, sh, cout, cin, wo, bo, U)
    _fails(chk._chk_fold_conv3x3, L.BF16, W, bias, s, sh, cout, cin, wo, bo, _bump(U, 5))
    bt = (bias.double().repeat(4) + K.view(4 * cout, cin).double() @ sh.double()).float()
    chk._chk_fold_tconv(L.BF16, K, bias, s, sh, cout, cin, (K.view(4 * cout, cin) * s).to(BF).view(-1), bt)
    _fails(chk._chk_fold_tconv, L.BF16, K, bias, s, sh, cout, cin, (K.view(4 * cout, cin)).to(BF).view(-1), bt)
    # column sums and border sums
    part = torch.randn(37 * 2 * 12, generator=g)
    out = part.view(37, 2, 12).double().sum((0, 1)).float()
    chk._chk_colsum(part, 37, 24, 2, out)
    _fails(chk._chk_colsum, part, 37, 24, 2, _bump(out))
    nn_, hh, ww, cc = 2, 5, 7, 8
    dz = torch.randn(nn_ * hh * ww * cc, generator=g).to(BF)
    d4 = dz.float().view(nn_, hh, ww, cc)
    bs = torch.stack([d4[:, 0].sum((0, 1)), d4[:, -1].sum((0, 1)), d4[:, :, 0].sum((0, 1)), d4[:, :, -1].sum((0, 1)),
                      d4[:, 0, 0].sum(0), d4[:, 0, -1].sum(0), d4[:, -1, 0].sum(0), d4[:, -1, -1].sum(0)])
    chk._chk_border_sums(L.BF16, dz, nn_, hh, ww, cc, bs.view(-1))
    _fails(chk._chk_border_sums, L.BF16, dz, nn_, hh, ww, cc, _bump(bs.view(-1), 20))


def _conv_v(db, bs, cout):
    """V[co][t] = db - the border sums of the pixels whose tap t falls outside (cnn_itmo.h mode 1)."""
    V = db.double()[:, None].repeat(1, 9)
    for t in range(9):
        r, q = divmod(t, 3)
        o = (r == 0) * bs[0] + (r == 2) * bs[1] + (q == 0) * bs[2] + (q == 2) * bs[3] \
            - (r == 0 and q == 0) * bs[4] - (r == 0 and q == 2) * bs[5] - (r == 2 and q == 0) * bs[6] \
            - (r == 2 and q == 2) * bs[7]
        V[:, t] -= o
    return V.reshape(-1)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_consumer_sums_check(mode):
    g = torch.Generator().manual_seed(5)
    cin_tot, ci0, c = 24, 8, 16
    cout = 3 if mode == 3 else 6
    K = cout * {1: 9, 2: 4, 3: 1}[mode]
    w, raw = torch.randn(K * cin_tot, generator=g), torch.randn(K * cin_tot, generator=g)
    db = torch.randn(cout, generator=g)
    vt = torch.randn(8 * cout, generator=g) if mode == 1 else torch.randn(4 * cout, generator=g) if mode == 2 else None
    V = _conv_v(db, vt.view(8, cout).double(), cout) if mode == 1 else vt.double() if mode == 2 else db.double()
    mean, inv = torch.rand(c, generator=g), torch.rand(c, generator=g) + .5
    Wm = w.view(K, cin_tot)[:, ci0:ci0 + c].double()
    Rm = raw.view(K, cin_tot)[:, ci0:ci0 + c].double()
    rows = L.CONSUMER_ROWS
    part = torch.zeros(rows, 2, c)
    for rr in range(rows):  # the kernel's grid row rr sums (co, tap) pairs [K*rr/rows, K*(rr+1)/rows)
        k0, k1 = K * rr // rows, K * (rr + 1) // rows
        swv, swr = (Wm[k0:k1] * V[k0:k1, None]).sum(0), (Wm[k0:k1] * Rm[k0:k1]).sum(0)
        part[rr, 0], part[rr, 1] = swv.float(), (inv.double() * (swr - mean.double() * swv)).float()
    chk = _checker(L.BF16)
    args = (mode, w, raw, cout, cin_tot, ci0, c, db, vt, mean, inv)
    chk._chk_bn_consumer_sums(*args, part.view(-1))
    j = int((part.view(-1).abs() > 1e-3).nonzero()[0])
    _fails(chk._chk_bn_consumer_sums, *args, _bump(part.view(-1), j))


@pytest.mark.parametrize("dt", [L.BF16, L.F32])
def test_fused_pool_checks(dt):
    """The fused-pool checks (cnnitmo_conv3x3_fwd_pool's pooled value and window index,
    cnnitmo_pool_bnsums_pooled): an emulation of the contract passes, a wrong index, a
    wrong value or a wrong sum fails.  Channel modes: max (+), min (-), first (0)."""
    T = BF if dt == L.BF16 else F32
    g = torch.Generator().manual_seed(3)
    n, h, w, c = 2, 6, 8, 16
    y = (torch.randint(0, 5, (n * h * w * c,), generator=g).float() / 4).to(T)  # many exact ties
    yv = View(y, n, h, w, c, c)
    sign = torch.tensor([1.0, -1.0, 0.0, 2.0] * 4)
    win = y.view(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 2, 4, 5).reshape(n, h // 2, w // 2, 4, c).double()
    key = win * torch.sign(sign).double()
    first = (key == key.max(3, keepdim=True).values).to(torch.uint8).argmax(3)
    pv = win.gather(3, first.unsqueeze(3)).squeeze(3).to(T).reshape(-1)
    pi = first.to(torch.uint8).reshape(-1)
    chk = _checker(dt)
    chk._chk_pool_of_stored("pool", dt, yv, pv, pi, sign)
    _fails(chk._chk_pool_of_stored, "pool", dt, yv, pv, (pi + 1) % 4, sign)
    _fails(chk._chk_pool_of_stored, "pool", dt, yv, _bump(pv), pi, sign)
    _fails(chk._chk_pool_of_stored, "pool", dt, yv, pv, pi, None)  # max everywhere: the min / first channels differ
    # pooled BN sums
    dyp = torch.randn(n * (h // 2) * (w // 2) * c, generator=g).to(T)
    mean, inv = torch.rand(c, generator=g), torch.rand(c, generator=g) + 0.5
    gd, pd = dyp.double().view(-1, c), pv.double().view(-1, c)
    part = torch.stack([gd.sum(0), (gd * (pd - mean.double()) * inv.double()).sum(0)]).float()[None]
    chk._chk_pool_bnsums_pooled(dt, dyp, pv, n, h, w, c, mean, inv, part)
    _fails(chk._chk_pool_bnsums_pooled, dt, dyp, pv, n, h, w, c, mean, inv, _bump(part, i=c + 2, by=1.0))


@pytest.mark.parametrize("dt", [L.BF16, L.F32])
def test_fused_head_check(dt):
    """cnnitmo_conv3x3_fwd_head's check: an fp32 evaluation of the contract (3x3 conv in fp32
    from dtype operands, ReLU, BN affine, the 1x1 head, sigmoid) passes; a value off by more
    than the fp32 slack fails, and so does a prediction of the unrounded conv with the affine
    left out."""
    T = BF if dt == L.BF16 else F32
    g = torch.Generator().manual_seed(5)
    n, h, w, cin, cout, hv = 2, 5, 7, 16, 64, 4
    x = torch.randn(n * h * w * cin, generator=g).to(T)
    wt = (torch.randn(cout * 9 * cin, generator=g) * 0.1).to(T)
    bias = torch.randn(cout, generator=g) * 0.1
    sc, sh = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.1
    hw, hb = torch.randn(3 * cout, generator=g) * 0.2, torch.randn(3, generator=g)
    xv = View(x, n, h, w, cin, cin)
    # fp32 evaluation: conv over fp32 operands, then the epilogue and the head in fp32
    xf = x.float().view(n, h, w, cin).permute(0, 3, 1, 2)
    wf = wt.float().view(cout, 3, 3, cin).permute(0, 3, 1, 2)
    z = torch.nn.functional.conv2d(xf, wf, bias, padding=1).permute(0, 2, 3, 1)
    y = torch.relu(z) * sc + sh
    yh = torch.sigmoid(y[:, :hv] @ hw.view(3, cout).t() + hb).contiguous()
    chk = _checker(dt)
    flags = L.RELU | L.AFFINE
    chk._chk_conv3x3_fwd_head(dt, xv, wt, bias, cout, flags, (sc, sh), hv, hw, hb, yh.view(-1))
    _fails(chk._chk_conv3x3_fwd_head, dt, xv, wt, bias, cout, flags, (sc, sh), hv, hw, hb, _bump(yh.view(-1), by=1e-3))
    y2 = torch.relu(z)
    yh2 = torch.sigmoid(y2[:, :hv] @ hw.view(3, cout).t() + hb).contiguous()
    _fails(chk._chk_conv3x3_fwd_head, dt, xv, wt, bias, cout, flags, (sc, sh), hv, hw, hb, yh2.view(-1))
