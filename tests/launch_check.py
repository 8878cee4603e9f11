"""Per-launch checker for full-size runs (test infrastructure, GPU only).

``LaunchChecker(ops, dt)`` wraps EVERY launching entry point of
``cnn_itmo_amd.ops`` so that, while the REAL engine runs a training step or an
inference forward at a benchmarked shape (BASELINE configs[1], [2], [4]), every
launch is verified the moment it returns, from the very buffers it read.  Each
check restates the entry point's contract in include/cnn_itmo.h and evaluates
it EXACTLY (fp64 on the GPU; torch GEMMs per image and tap for the convolutions
-- an independent vendor path) over the WHOLE output of the launch:

* conv3x3 / tconv2x2 / first-layer forwards: bias, folded-BN border correction,
  ReLU, inference affine; their BN partial sums (STATS) against the exact
  per-channel sums;
* input gradients, incl. the fused ``*_dgrad_bn`` launches' producer BN backward
  dz = [r>0]*(a*bf16(g) - b*r + e) and their column partials;
* weight gradients, incl. the folded-BN correction (the reference differentiates
  w.r.t. the conv's true input y = r*s + h) and the raw (uncorrected) sums;
* every launch that is not a GEMM (pooling, BatchNormalization forward and
  backward in all their forms, Dropout, the sigmoid/MSE/accuracy head, RMSprop,
  weight preparation and BN folding): ``launch_check_elem.py``.

Coverage is enforced, not assumed: the checker also wraps ``ops.call`` and
records any library call made outside a checked entry point
(``LaunchChecker.unchecked``); the tests assert that set is empty.

Tolerances: bf16 stores within 1.01*2^-8*|exact| + 2^-12*max|exact| (round-to-nearest
of an fp32 accumulation); fp32 stores within 1e-5*|exact| + 1e-6*max|exact| + 8*2^-24*sqrt(K)*sum|w*x|;
partial sums within 1e-5 of the channel's sum of |values|; weight gradients
rel-L2 <= 1e-3 (bf16 inputs) / 1e-5 (fp32); the non-GEMM checks state theirs in
launch_check_elem.py.
"""
from __future__ import annotations

import time

import torch

from cnn_itmo_amd import _lib as L
from launch_check_elem import ElementwiseChecks

F64 = torch.float64
BF = torch.bfloat16


def _conv3(x3, W, hv=None):
    """Exact 'same' 3x3 conv of one image: x3 [h,w,cin] (any dtype) and W
    [cout,3,3,cin] -> fp64 [h,w,cout] (rows >= hv of x3 read as zero)."""
    h, w, cin = x3.shape
    xd = x3.to(F64)
    if hv is not None and hv < h:
        xd = xd.clone()
        xd[hv:] = 0
    xp = torch.nn.functional.pad(xd, (0, 0, 1, 1, 1, 1))
    Wd = W.to(F64)
    z = None
    for r in range(3):
        for s in range(3):
            t = xp[r:r + h, s:s + w] @ Wd[:, r, s].t()
            z = t if z is None else z + t
    return z


def _atb(d, y, chunk=8192):
    """d^T @ y for tall d [P, a], y [P, b] (fp64) as a batched split-K GEMM: a single
    GEMM with K = P ~ 2M and a, b <= 768 runs on a handful of workgroups."""
    P = d.shape[0]
    nc = -(-P // chunk)
    pad = nc * chunk - P
    if pad:
        d = torch.nn.functional.pad(d, (0, 0, 0, pad))
        y = torch.nn.functional.pad(y, (0, 0, 0, pad))
    return torch.bmm(d.reshape(nc, chunk, -1).transpose(1, 2), y.reshape(nc, chunk, -1)).sum(0)


def _border_map(U, h, w, dev):
    """[h, w, cout] folded-BN zero-padding correction (igemm_common.h border_corr)."""
    U = U.view(-1, 8).to(F64)
    oh = torch.arange(h, device=dev)[:, None, None]
    ow = torch.arange(w, device=dev)[None, :, None]
    top, bot, lef, rig = oh == 0, oh == h - 1, ow == 0, ow == w - 1
    return (top * U[:, 0] + bot * U[:, 1] + lef * U[:, 2] + rig * U[:, 3]
            - (top & lef) * U[:, 4] - (top & rig) * U[:, 5] - (bot & lef) * U[:, 6] - (bot & rig) * U[:, 7])


def _epilogue(z, flags, aff):
    if flags & L.RELU:
        z = z.clamp_min(0)
    if flags & L.AFFINE:
        z = z * aff[0].to(F64) + aff[1].to(F64)
    return z


def _f32_slack(dt, K, absconv):
    """fp32 accumulation slack: 8 * 2^-24 * sqrt(K) * sum_k |w_k x_k| (None for bf16, whose
    output rounding dominates)."""
    return None if dt == L.BF16 else 8 * 2.0 ** -24 * (K ** 0.5) * absconv


class _Acc:
    """Streams per-image comparisons of one launch into one worst-case figure."""

    def __init__(self, chk, label, dt=None):
        self.chk, self.label = chk, label
        self.dt = chk.dt if dt is None else dt
        self.pairs = []

    def add(self, got, ref, extra=None):
        self.pairs.append((got, ref.to(F64), extra))

    def done(self):
        scale = max(float(r.abs().max()) for _, r, _ in self.pairs) if self.pairs else 0.0
        scale = max(scale, 1e-30)
        worst, maxerr = 0.0, 0.0
        for got, ref, extra in self.pairs:
            if self.dt == L.BF16:
                bound = 2.0 ** -8 * 1.01 * ref.abs() + 2.0 ** -12 * scale
            else:
                bound = 1e-5 * ref.abs() + 1e-6 * scale
            if extra is not None:
                bound = bound + extra
            err = (got.to(F64) - ref).abs()
            worst = max(worst, float((err / bound).max()))
            maxerr = max(maxerr, float(err.max()))
        self.chk.log.append((self.label, "err/bound", worst))
        assert worst <= 1.0, f"{self.label}: max |got-exact|/bound = {worst:.3f} (max err {maxerr:.3e}, scale {scale:.3e})"


# every launching entry point of cnn_itmo_amd.ops (all of them go through ops.call)
LAUNCHES = ("conv3x3_fwd", "conv3x3_fwd_pool", "conv3x3_fwd_head", "pool_bnsums_pooled", "conv3x3_fwd_cat", "conv_wgrad_cat", "conv3x3_dgrad", "conv3x3_dgrad_bn", "conv3x3_dgrad_bn_pooled", "tconv_fwd", "tconv_dgrad",
            "tconv_dgrad_bn", "conv_wgrad", "tconv_wgrad", "conv_c3_fwd", "conv_c3_wgrad", "conv1tap_fwd", "im2col_c3",
            "maxpool_fwd", "maxpool_bwd", "pool_bnsums", "bn_fwd_finalize", "bn_infer_coeffs", "bn_apply",
            "bn_bwd_reduce", "bn_bwd_finalize", "bn_bwd_apply", "bn_bwd_apply_pooled", "bn_bwd_apply_g3",
            "bn_consumer_sums", "colsum", "border_sums", "head_fwd", "head_fwd_bwd", "head_fwd_bwd_g3",
            "head_finalize", "rmsprop", "prep_conv3x3", "prep_tconv", "prep_c3", "fold_conv3x3", "fold_tconv")


class LaunchChecker(ElementwiseChecks):
    def __init__(self, ops, dt, verbose=True):
        self.ops, self.dt, self.verbose = ops, dt, verbose
        self.log = []   # (launch label, metric, value)
        self.orig = {}
        self.calls = {}  # entry point -> checked launches
        self.unchecked = {}  # library symbol -> calls made outside a checked entry point
        self._depth = 0
        for nm in LAUNCHES:
            self.orig[nm] = getattr(ops, nm)
            setattr(ops, nm, self._wrap(nm))
        self.orig["call"] = ops.call
        lib_call = ops.call

        def call(name, *a):
            if self._depth == 0:
                self.unchecked[name] = self.unchecked.get(name, 0) + 1
            return lib_call(name, *a)
        ops.call = call

    def restore(self):
        for nm, f in self.orig.items():
            setattr(self.ops, nm, f)

    def _acc(self, label, dt=None):
        return _Acc(self, label, dt)

    def _wrap(self, nm):
        orig, chk = self.orig[nm], getattr(self, "_chk_" + nm)
        pre = getattr(self, "_pre_" + nm, None)

        def f(*a, **k):
            snap = None
            if pre is not None:  # in-place operands: their state before the launch
                torch.cuda.synchronize()
                snap = pre(*a, **k)
            self._depth += 1
            try:
                r = orig(*a, **k)
            finally:
                self._depth -= 1
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n0 = len(self.log)
            if pre is not None:
                chk(*a, pre=snap, **k)
            else:
                chk(*a, **k)
            self.calls[nm] = self.calls.get(nm, 0) + 1
            if self.verbose:  # progress: one line per checked launch
                worst = ", ".join(f"{m} {v:.2e}" for _, m, v in self.log[n0:])
                lab = self.log[n0][0] if len(self.log) > n0 else nm
                print(f"[check {time.perf_counter() - t0:5.1f}s] {lab}: {worst}", flush=True)
            return r
        return f

    # ---- tolerances ------------------------------------------------------------------
    def _close_full(self, label, got, ref):
        got, ref = got.to(F64).reshape(-1), ref.to(F64).reshape(-1)
        rel = float((got - ref).norm() / max(1e-30, float(ref.norm())))
        mx = float((got - ref).abs().max() / max(1e-30, float(ref.abs().max())))
        tl, tm = (1e-3, 5e-3) if self.dt == L.BF16 else (1e-5, 1e-4)
        self.log.append((label, "rel-L2", rel))
        assert rel <= tl and mx <= tm, f"{label}: rel-L2 {rel:.3e} (<= {tl}), max-abs/max {mx:.3e} (<= {tm})"

    def _sums(self, label, got, exact, absum):
        """Partial-sum totals vs exact sums (fp32 partials of <= 256 values, fp64 fold)."""
        worst = float(((got - exact).abs() / (1e-5 * absum + 1e-12)).max())
        self.log.append((label, "sum err/bound", worst))
        assert worst <= 1.0, f"{label}: partial-sum totals off ({worst:.2f} x bound)"

    # ---- conv3x3 -------------------------------------------------------------------
    def _chk_conv3x3_fwd(self, dt, x, wt, bias, out, flags=0, aff=None, stats=None, border=None, tag=""):
        n, h, w, cin, cout = x.n, x.h, x.w, x.c, out.c
        lab = f"conv3x3_fwd{tag} {n}x{h}x{w} {cin}->{cout}"
        W = wt.view(cout, 3, 3, cin)
        bmap = _border_map(border, h, w, wt.device) if border is not None else 0
        acc = _Acc(self, lab)
        s1 = torch.zeros(cout, dtype=F64, device=wt.device)
        s2, sa, sa2 = torch.zeros_like(s1), torch.zeros_like(s1), torch.zeros_like(s1)
        xt, ot = x.tensor(), out.tensor()
        for i in range(n):
            z = _conv3(xt[i], W) + (bias.to(F64) if bias is not None else 0) - bmap
            sl = None
            if self.dt != L.BF16:
                sl = _f32_slack(self.dt, 9 * cin, _conv3(xt[i].abs(), W.abs()))
                if flags & L.AFFINE:
                    sl = sl * aff[0].to(F64).abs()
            z = _epilogue(z, flags, aff)
            acc.add(ot[i], z, sl)
            if stats is not None:
                s1 += z.sum((0, 1))
                s2 += (z * z).sum((0, 1))
                sa += z.abs().sum((0, 1))
                sa2 += (z * z).sum((0, 1))
        acc.done()
        if stats is not None and flags & L.STATS:
            tot = stats.view(-1, 2, cout).to(F64).sum(0)
            self._sums(lab + " stats", tot[0], s1, sa)
            self._sums(lab + " stats^2", tot[1], s2, sa2)

    def _chk_conv3x3_fwd_pool(self, dt, x, wt, bias, out, pool_out, pool_idx, pool_sign=None, flags=0, aff=None,
                              stats=None, border=None):
        self._chk_conv3x3_fwd(dt, x, wt, bias, out, flags, aff, stats, border, tag="_pool")
        self._chk_pool_of_stored(f"conv3x3_fwd_pool {x.n}x{x.h}x{x.w} {x.c}->{out.c}", dt, out, pool_out, pool_idx,
                                 pool_sign)

    def _chk_conv3x3_fwd_head(self, dt, x, wt, bias, cout, flags, aff, h_valid, head_w, head_b, yhat):
        """yhat = sigmoid(epilogue(conv) . head_w^T + head_b) over the valid rows; the conv is
        accumulated in fp32 from operands in dtype and never rounded to dtype, so the bound is
        the fp32 accumulation slack carried through the head's weights, plus the head's own
        fp32 dot product, times the sigmoid's slope (<= 1/4)."""
        n, h, w, cin = x.n, x.h, x.w, x.c
        lab = f"conv3x3_fwd_head {n}x{h}x{w} {cin}->{cout}->3 (valid {h_valid})"
        W = wt.view(cout, 3, 3, cin)
        Hw, hb = head_w.view(3, cout).to(F64), head_b.to(F64)
        yt, xt = yhat.view(n, h_valid, w, 3), x.tensor()
        sc = aff[0].to(F64).abs() if (flags & L.AFFINE) else 1.0
        for i in range(n):
            y = _epilogue(_conv3(xt[i], W) + bias.to(F64), flags, aff)[:h_valid]
            sl = (_f32_slack(L.F32, 9 * cin, _conv3(xt[i].abs(), W.abs())) * sc)[:h_valid]
            z = y @ Hw.t() + hb
            dz = sl @ Hw.abs().t() + 16 * 2.0 ** -24 * (y.abs() @ Hw.abs().t() + hb.abs())
            self._close(lab, yt[i], torch.sigmoid(z), 0.25 * dz + 1e-7)

    @staticmethod
    def _cat_view(x1, x2):
        """The concatenate [x1, x2] (channels) as one dense View (a copy; test only)."""
        t = torch.cat([x1.tensor(), x2.tensor()], dim=3).contiguous()
        from cnn_itmo_amd.ops import View
        return View(t.view(-1), x1.n, x1.h, x1.w, x1.c + x2.c, x1.c + x2.c, 0)

    def _chk_conv3x3_fwd_cat(self, dt, x1, x2, wt, bias, out, flags=0, aff=None, stats=None, border=None):
        self._chk_conv3x3_fwd(dt, self._cat_view(x1, x2), wt, bias, out, flags, aff, stats, border, tag="_cat")

    def _chk_conv_wgrad_cat(self, dt, x1, x2, dz, cout, dw, fold=None, raw=None):
        self._chk_conv_wgrad(dt, 9, self._cat_view(x1, x2), dz, cout, dw, fold=fold, raw=raw, tag="_cat")

    def _chk_conv3x3_dgrad(self, dt, dz, n, h, w, cout, wflip, cin, dx):
        d4, Wf, dxt = dz.view(n, h, w, cout), wflip.view(-1)[:cin * 9 * cout].view(cin, 3, 3, cout), dx.tensor()
        acc = _Acc(self, f"conv3x3_dgrad {n}x{h}x{w} {cout}->{cin}")
        for i in range(n):
            acc.add(dxt[i], _conv3(d4[i], Wf))
        acc.done()

    def _bnb_ref(self, g, r, coef, c):
        """dz = [r>0]*(a*bf16(g) - b*r + e) and the slack for one bf16 ulp of g flipping
        between the exact g and the kernel's fp32 accumulation."""
        a, b, e = coef.view(3, c).to(F64)
        gb = g.to(BF).to(F64) if self.dt == L.BF16 else g
        rd = r.to(F64)
        ref = torch.where(rd > 0, a * gb - b * rd + e, torch.zeros_like(gb))
        extra = 2.0 ** -7 * (a * g).abs() if self.dt == L.BF16 else None
        return ref, extra

    @staticmethod
    def _rtensor(r, n, h, w, c):
        return r.view(n, h, w, c) if isinstance(r, torch.Tensor) else r.tensor()

    def _chk_conv3x3_dgrad_bn(self, dt, dz, n, h, w, cout, wflip, cin, dx, c0, c1, coef, r, dz_out, part, parity):
        c = c1 - c0
        lab = f"conv3x3_dgrad_bn {n}x{h}x{w} {cout}->{cin} [{c0},{c1})"
        d4, Wf = dz.view(n, h, w, cout), wflip.view(-1)[:cin * 9 * cout].view(cin, 3, 3, cout)
        rt, zo = self._rtensor(r, n, h, w, c), dz_out.view(n, h, w, c)
        dxt = dx.tensor() if dx is not None else None
        acc, accx = _Acc(self, lab), _Acc(self, lab + " dx")
        npar = 4 if parity else 1
        ps = torch.zeros(npar, c, dtype=F64, device=dz.device)
        pa = torch.zeros_like(ps)
        for i in range(n):
            g = _conv3(d4[i], Wf)
            ref, extra = self._bnb_ref(g[..., c0:c1], rt[i], coef, c)
            acc.add(zo[i], ref, extra)
            if dxt is not None and (c0 > 0 or c1 < cin):
                keep = torch.ones(cin, dtype=torch.bool, device=dz.device)
                keep[c0:c1] = False
                accx.add(dxt[i][..., keep], g[..., keep])
            zs = zo[i].to(F64)  # the partials sum the stored (rounded) dz
            for ph in range(2 if parity else 1):
                for pw in range(2 if parity else 1):
                    v = zs[ph::2, pw::2] if parity else zs
                    ps[ph * 2 + pw if parity else 0] += v.sum((0, 1))
                    pa[ph * 2 + pw if parity else 0] += v.abs().sum((0, 1))
        acc.done()
        if accx.pairs:
            accx.done()
        tot = part.view(-1, npar, c).to(F64).sum(0)
        self._sums(lab + " part", tot, ps, pa)

    def _chk_conv3x3_dgrad_bn_pooled(self, dt, dz, n, h, w, cout, wflip, cin, coef, r, dyp, idx, dz_out, part):
        """dz = [r>0]*(a*(bf16(g) + routed) - b*r + e): g the exact skip-path input gradient,
        routed = the pooled gradient at the window position its index byte names."""
        lab = f"conv3x3_dgrad_bn_pooled {n}x{h}x{w} {cout}->{cin}"
        d4, Wf = dz.view(n, h, w, cout), wflip.view(-1)[:cin * 9 * cout].view(cin, 3, 3, cout)
        rt, zo = self._rtensor(r, n, h, w, cin), dz_out.view(n, h, w, cin)
        gp, ix = dyp.view(n, h // 2, w // 2, cin), idx.view(n, h // 2, w // 2, cin)
        a, b, e = coef.view(3, cin).to(F64)
        acc = _Acc(self, lab)
        ps = torch.zeros(1, cin, dtype=F64, device=dz.device)
        pa = torch.zeros_like(ps)
        for i in range(n):
            g = _conv3(d4[i], Wf)
            routed = torch.zeros_like(g)
            gpi, ixi = gp[i].to(F64), ix[i]
            for k in range(4):
                routed[k // 2::2, k % 2::2] = torch.where(ixi == k, gpi, torch.zeros_like(gpi))
            gb = (g.to(BF).to(F64) if self.dt == L.BF16 else g) + routed
            rd = rt[i].to(F64)
            ref = torch.where(rd > 0, a * gb - b * rd + e, torch.zeros_like(gb))
            extra = 2.0 ** -7 * (a * g).abs() if self.dt == L.BF16 else None
            acc.add(zo[i], ref, extra)
            ps[0] += zo[i].to(F64).sum((0, 1))
            pa[0] += zo[i].to(F64).abs().sum((0, 1))
        acc.done()
        self._sums(lab + " part", part.view(-1, 1, cin).to(F64).sum(0), ps, pa)

    def _chk_conv_wgrad(self, dt, ntaps, x, dz, cout, dw, dw_cols=0, fold=None, raw=None, tag=""):
        n, h, w, cin = x.n, x.h, x.w, x.c
        lab = f"conv_wgrad{tag}({ntaps}) {n}x{h}x{w} {cin}->{cout}"
        xt, d4 = x.tensor(), dz.view(n, h, w, cout)
        if ntaps == 1:  # im2col columns (fp32 first layer): dw [cout][dw_cols or cin]
            kc = dw_cols or cin
            ref = torch.zeros(cout, kc, dtype=F64, device=dz.device)
            for i in range(n):
                ref += _atb(d4[i].reshape(-1, cout).to(F64), xt[i].reshape(-1, cin)[:, :kc].to(F64))
            self._close_full(lab, dw.view(cout, kc), ref)
            return
        ref = torch.zeros(cout, 3, 3, cin, dtype=F64, device=dz.device)
        rawr = torch.zeros_like(ref) if raw is not None else None
        for i in range(n):
            d = d4[i].reshape(-1, cout).to(F64)
            rpad = torch.nn.functional.pad(xt[i].to(F64), (0, 0, 1, 1, 1, 1))
            ypad = (torch.nn.functional.pad(xt[i].to(F64) * fold[0].to(F64) + fold[1].to(F64), (0, 0, 1, 1, 1, 1))
                    if fold is not None else rpad)
            for r in range(3):
                for q in range(3):
                    ref[:, r, q] += _atb(d, ypad[r:r + h, q:q + w].reshape(-1, cin))
                    if rawr is not None:
                        rawr[:, r, q] += _atb(d, rpad[r:r + h, q:q + w].reshape(-1, cin))
        self._close_full(lab + (" (folded)" if fold is not None else ""), dw.view(cout, 3, 3, cin), ref)
        if rawr is not None:
            self._close_full(lab + " raw", raw.view(cout, 3, 3, cin), rawr)

    # ---- first layer -----------------------------------------------------------------
    def _c3_input(self, x, n, hv, h, w, dt):
        """[n, h, w, 3] input as the kernel sees it (bf16 cast when dt is bf16, zero rows >= hv)."""
        xp = x.view(n, hv, w, 3)
        if dt == L.BF16:
            xp = xp.to(BF)
        return torch.nn.functional.pad(xp.to(F64), (0, 0, 0, 0, 0, h - hv))

    def _chk_conv_c3_fwd(self, dt, x, n, hv, h, w, wt, bias, out, flags=0, aff=None, stats=None):
        xin = self._c3_input(x, n, hv, h, w, dt)
        W = wt.view(32, 32)[:, :27].reshape(32, 3, 3, 3)
        lab = f"conv_c3_fwd {n}x{h}x{w} (valid {hv})"
        acc, ot = _Acc(self, lab, dt), out.tensor()
        s1 = torch.zeros(32, dtype=F64, device=x.device)
        sa = torch.zeros_like(s1)
        for i in range(n):
            z = _epilogue(_conv3(xin[i], W) + bias.to(F64), flags, aff)
            sl = _f32_slack(dt, 27, _conv3(xin[i].abs(), W.abs()))
            if sl is not None and flags & L.AFFINE:
                sl = sl * aff[0].to(F64).abs()
            acc.add(ot[i], z, sl)
            s1 += z.sum((0, 1))
            sa += z.abs().sum((0, 1))
        acc.done()
        if stats is not None and flags & L.STATS:
            tot = stats.view(-1, 2, 32).to(F64).sum(0)
            self._sums(lab + " stats", tot[0], s1, sa)

    def _chk_conv_c3_wgrad(self, dt, x, n, hv, h, w, dz, dw):
        xin = self._c3_input(x, n, hv, h, w, dt)
        d4 = dz.view(n, h, w, 32)
        ref = torch.zeros(32, 3, 3, 3, dtype=F64, device=dz.device)
        for i in range(n):
            d = d4[i].reshape(-1, 32).to(F64)
            xq = torch.nn.functional.pad(xin[i], (0, 0, 1, 1, 1, 1))
            for r in range(3):
                for q in range(3):
                    ref[:, r, q] += _atb(d, xq[r:r + h, q:q + w].reshape(-1, 3))
        self._close_full(f"conv_c3_wgrad {n}x{h}x{w}", dw.view(32, 3, 3, 3), ref)

    def _chk_im2col_c3(self, dt, x, n, hv, h, w, cols):
        xin = self._c3_input(x, n, hv, h, w, dt)
        c4 = cols.view(n, h, w, 32)
        acc = _Acc(self, f"im2col_c3 {n}x{h}x{w}")
        for i in range(n):
            xp = torch.nn.functional.pad(xin[i], (0, 0, 1, 1, 1, 1))
            ref = torch.stack([xp[r:r + h, s:s + w] for r in range(3) for s in range(3)], 2).reshape(h, w, 27)
            acc.add(c4[i][..., :27], ref)
            assert float(c4[i][..., 27:].abs().max()) == 0.0
        acc.done()

    def _chk_conv1tap_fwd(self, dt, cols, k, m, wt, bias, out, flags=0, aff=None, stats=None):
        A = cols.view(m, k)
        got = out.buf.view(-1)[out.off:].as_strided((m, out.c), (out.ld, 1))
        acc = _Acc(self, f"conv1tap_fwd m={m}")
        Wd = wt.view(-1, k).to(F64).t()
        step = 1 << 22
        for a in range(0, m, step):
            b = min(m, a + step)
            sl = _f32_slack(self.dt, k, A[a:b].to(F64).abs() @ Wd.abs())
            if sl is not None and flags & L.AFFINE:
                sl = sl * aff[0].to(F64).abs()
            acc.add(got[a:b], _epilogue(A[a:b].to(F64) @ Wd + bias.to(F64), flags, aff), sl)
        acc.done()

    # ---- Conv2DTranspose ---------------------------------------------------------------
    def _chk_tconv_fwd(self, dt, x, k, bias, out, flags=0, aff=None, stats=None):
        n, h, w, cin, cout = x.n, x.h, x.w, x.c, out.c
        lab = f"tconv_fwd {n}x{h}x{w} {cin}->{cout}"
        K = k.view(2, 2, cout, cin).to(F64)
        bb = bias.to(F64).view(4, cout) if (bias is not None and flags & L.BIAS_PER_COL) else None
        acc = _Acc(self, lab)
        xt, o6 = x.tensor(), out.tensor().view(n, h, 2, w, 2, cout)
        s1 = torch.zeros(4, cout, dtype=F64, device=k.device)
        s2, sa, sa2 = torch.zeros_like(s1), torch.zeros_like(s1), torch.zeros_like(s1)
        for i in range(n):
            xi = xt[i].to(F64)
            for a in range(2):
                for b in range(2):
                    z = xi @ K[a, b].t()
                    sl = _f32_slack(self.dt, cin, xi.abs() @ K[a, b].abs().t())
                    if sl is not None and flags & L.AFFINE:
                        sl = sl * aff[0].to(F64).abs()
                    if bias is not None:
                        z = z + (bb[a * 2 + b] if bb is not None else bias.to(F64))
                    z = _epilogue(z, flags, aff)
                    acc.add(o6[i, :, a, :, b], z, sl)
                    if stats is not None:
                        t = a * 2 + b
                        s1[t] += z.sum((0, 1))
                        s2[t] += (z * z).sum((0, 1))
                        sa[t] += z.abs().sum((0, 1))
                        sa2[t] += (z * z).sum((0, 1))
        acc.done()
        if stats is not None and flags & L.STATS:
            # contract: per-channel totals over the 4 tap column groups (bn_fwd_finalize
            # folds the groups; tconv_ws's 256-column block puts both of its taps' sums in
            # the first tap's columns)
            tot = stats.view(-1, 2, 4, cout).to(F64).sum(0).sum(1)
            self._sums(lab + " stats", tot[0], s1.sum(0), sa.sum(0))
            self._sums(lab + " stats^2", tot[1], s2.sum(0), sa2.sum(0))

    @staticmethod
    def _tdgrad(d6i, kt):
        """input gradient of one image: d6i [h,2,w,2,cout], kt [cin,2,2,cout] -> [h,w,cin]."""
        g = None
        for a in range(2):
            for b in range(2):
                t = d6i[:, a, :, b].to(F64) @ kt[:, a, b].t()
                g = t if g is None else g + t
        return g

    def _chk_tconv_dgrad(self, dt, dout, n, h, w, cout, kT, cin, dx):
        d6, kt = dout.view(n, h, 2, w, 2, cout), kT.view(cin, 2, 2, cout).to(F64)
        acc = _Acc(self, f"tconv_dgrad {n}x{h}x{w} {cout}->{cin}")
        for i in range(n):
            acc.add(dx.view(n, h, w, cin)[i], self._tdgrad(d6[i], kt))
        acc.done()

    def _chk_tconv_dgrad_bn(self, dt, dout, n, h, w, cout, kT, cin, coef, r, dz_out, part):
        lab = f"tconv_dgrad_bn {n}x{h}x{w} {cout}->{cin}"
        d6, kt = dout.view(n, h, 2, w, 2, cout), kT.view(cin, 2, 2, cout).to(F64)
        rt, zo = self._rtensor(r, n, h, w, cin), dz_out.view(n, h, w, cin)
        acc = _Acc(self, lab)
        ps = torch.zeros(1, cin, dtype=F64, device=dout.device)
        pa = torch.zeros_like(ps)
        for i in range(n):
            ref, extra = self._bnb_ref(self._tdgrad(d6[i], kt), rt[i], coef, cin)
            acc.add(zo[i], ref, extra)
            ps[0] += zo[i].to(F64).sum((0, 1))
            pa[0] += zo[i].to(F64).abs().sum((0, 1))
        acc.done()
        self._sums(lab + " part", part.view(-1, 1, cin).to(F64).sum(0), ps, pa)

    def _chk_tconv_wgrad(self, dt, x, dout, cout, dk, fold=None, raw=None):
        n, h, w, cin = x.n, x.h, x.w, x.c
        xt, d6 = x.tensor(), dout.view(n, h, 2, w, 2, cout)
        ref = torch.zeros(2, 2, cout, cin, dtype=F64, device=dout.device)
        rawr = torch.zeros_like(ref) if raw is not None else None
        for i in range(n):
            r2 = xt[i].reshape(-1, cin).to(F64)
            y2 = r2 * fold[0].to(F64) + fold[1].to(F64) if fold is not None else r2
            for a in range(2):
                for b in range(2):
                    d = d6[i, :, a, :, b].reshape(-1, cout).to(F64)
                    ref[a, b] += _atb(d, y2)
                    if rawr is not None:
                        rawr[a, b] += _atb(d, r2)
        lab = f"tconv_wgrad {n}x{h}x{w} {cin}->{cout}"
        self._close_full(lab + (" (folded)" if fold is not None else ""), dk.view(2, 2, cout, cin), ref)
        if rawr is not None:
            self._close_full(lab + " raw", raw.view(2, 2, cout, cin), rawr)

    def summary(self):
        seen = {}
        for lab, met, v in self.log:
            seen[(lab, met)] = max(seen.get((lab, met), 0.0), v)
        return seen
