"""Per-launch checks of every launch that is not a GEMM (test infrastructure, GPU only).

Mixed into ``launch_check.LaunchChecker``.  Each ``_chk_<op>`` restates the contract
of one entry point of include/cnn_itmo.h and evaluates it in fp64 on the GPU over
the WHOLE output of the launch, from the very buffers it read (in-place operands
are snapshotted by the matching ``_pre_<op>`` before the launch):

* MaxPooling2D forward / backward (model.py:210,215,220,227): argmax bytes under
  the first-max rule -- bit-exact on raw inputs, and on a folded BN input (the
  pool sees r*s + h formed in fp32) every deviation from the fp64 first-max must
  be a tie within the fp32 rounding of that affine; the backward scatter-add
  bit-exact (one fp32 add, round to nearest even);
* BatchNormalization (model.py:196,200): the forward finalize (batch mean,
  biased variance, scale/shift, Keras-2.2 moving statistics with both Bessel
  factors), inference coefficients, the materialised BN + Dropout(0.5) apply
  (model.py:226,239; counter-hash mask reproduced bit for bit), the backward
  reduce / finalize / apply in its plain, parity, Dropout, pooled-route and
  rank-3 (head g3) forms, the MaxPooling2D share of the sums, the consumer-derived
  sums, border sums and column reductions;
* the sigmoid head + MSE + categorical accuracy (model.py:276,281): g3, loss,
  correct count, db, dW partials and their finalize;
* RMSprop (model.py:281) over the whole flat parameter buffer;
* the per-step weight preparation and BN folding (bit-exact casts / layouts).

Tolerances (stated per check below): bf16 stores within round-to-nearest of the
fp32 value plus the fp32 evaluation error; fp32 results within a few ulp of the
fp64 restatement; partial-sum totals within 1e-5 of the sum of |terms| (plus the
sum of the per-element bounds where the terms themselves carry rounding).
"""
from __future__ import annotations

import numpy as np
import torch

from cnn_itmo_amd import _lib as L

F64 = torch.float64
BF = torch.bfloat16
U32 = 2.0 ** -23  # fp32 ulp (relative)


# ---- Dropout(0.5) counter hash (common.h dropout_keep, oracle/unet_ref.py:dropout_keep)
def _s64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def _lsr(x, k):
    """logical right shift of an int64 tensor holding uint64 bits"""
    return (x >> k) & ((1 << (64 - k)) - 1)


_G1, _G2 = 0x9E3779B97F4A7C15, 0xD1B54A32D192ED03
_M1, _M2 = _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)


def dropout_keep(seed, layer, idx):
    """keep mask for int64 element indices idx (two's-complement wrap = uint64 arithmetic)."""
    x = idx + _s64(int(seed) * _G1 + int(layer) * _G2)
    x = x ^ _lsr(x, 30)
    x = x * _M1
    x = x ^ _lsr(x, 27)
    x = x * _M2
    x = x ^ _lsr(x, 31)
    return x >= 0


def _tdt(dt):
    return BF if dt == L.BF16 else torch.float32


def _f32(v):
    return float(np.float32(v))


class ElementwiseChecks:
    """Mixin: needs self.log (list), self._acc(label, dt) and self._sums(label, got, exact, absum)."""

    # ---- helpers --------------------------------------------------------------------
    def _close(self, label, got, ref, bound):
        """|got - ref| <= bound elementwise (all fp64 tensors of one shape)."""
        got = got.to(F64)
        err = (got - ref).abs()
        r = float((err / bound.clamp_min(1e-300)).max()) if err.numel() else 0.0
        self.log.append((label, "err/bound", r))
        assert r <= 1.0, f"{label}: max |got-ref|/bound = {r:.3f} (max err {float(err.max()):.3e})"

    def _exact(self, label, ok, what="bit-exact"):
        bad = int((~ok).sum())
        self.log.append((label, what + " mismatches", float(bad)))
        assert bad == 0, f"{label}: {bad} elements differ ({what})"

    @staticmethod
    def _img(t, i, n):
        """rows of image i of a [p][c] tensor holding n images"""
        hw = t.shape[0] // n
        return t[i * hw:(i + 1) * hw]

    # ---- MaxPooling2D ---------------------------------------------------------------
    def _chk_maxpool_fwd(self, dt, x, y, idx, aff=None):
        n, h, w, c = x.n, x.h, x.w, x.c
        ho, wo = h // 2, w // 2
        lab = f"maxpool_fwd {n}x{h}x{w}x{c}" + (" (folded BN)" if aff is not None else "")
        xt, y4, i4 = x.tensor(), y.view(n, ho, wo, c), idx.view(n, ho, wo, c)
        acc = self._acc(lab, dt)
        mism = ties = 0
        for i in range(n):
            r = xt[i, :2 * ho, :2 * wo].to(F64)
            if aff is not None:
                s, sh = aff[0].to(F64), aff[1].to(F64)
                v = r * s + sh
                tol = 4 * U32 * ((r * s).abs() + sh.abs())  # fp32 evaluation of r*s + h
            else:
                v = r
            win = v.view(ho, 2, wo, 2, c).permute(0, 2, 1, 3, 4).reshape(ho, wo, 4, c)
            mx = win.max(2).values
            first = (win == mx.unsqueeze(2)).to(torch.uint8).argmax(2)  # first maximum, window order
            got = i4[i].long()
            assert int(got.max()) <= 3, f"{lab}: argmax byte > 3"
            if aff is None:  # raw inputs: bit-exact, tie rule included
                self._exact(lab + " idx", got == first)
                self._exact(lab + " y", y4[i].to(F64) == mx)
                continue
            acc.add(y4[i], mx)
            tw = tol.view(ho, 2, wo, 2, c).permute(0, 2, 1, 3, 4).reshape(ho, wo, 4, c).amax(2)
            sel = win.gather(2, got.unsqueeze(2)).squeeze(2)
            ok = sel >= mx - 2 * tw  # the chosen element is a maximum up to rounding
            for k in range(3):  # every element before the chosen one is strictly smaller up to rounding
                ok &= ~((got > k) & (win[:, :, k] >= sel + 2 * tw))
            self._exact(lab + " idx (first-max up to fp32 ties)", ok, "rule")
            d = got != first
            mism += int(d.sum())
            srt = win.sort(2, descending=True).values
            ties += int(((srt[:, :, 0] - srt[:, :, 1]) <= 2 * tw).sum())
        if aff is not None:
            acc.done()
            self.log.append((lab, "argmax != fp64 first-max (near ties)", float(mism)))
            assert mism <= ties, f"{lab}: {mism} argmax mismatches but only {ties} near ties"

    def _pre_maxpool_bwd(self, dt, dy, idx, dx):
        return dx.tensor().clone()

    def _chk_maxpool_bwd(self, dt, dy, idx, dx, pre=None):
        n, h, w, c = dx.n, dx.h, dx.w, dx.c
        ho, wo = h // 2, w // 2
        lab = f"maxpool_bwd {n}x{h}x{w}x{c}"
        after, d4, i4 = dx.tensor(), dy.view(n, ho, wo, c), idx.view(n, ho, wo, c)
        T = _tdt(dt)
        for i in range(n):
            b = pre[i].float()
            add = torch.zeros_like(b)
            a6 = add[:2 * ho, :2 * wo].view(ho, 2, wo, 2, c)
            hit = torch.zeros(b.shape, dtype=torch.bool, device=b.device)
            h6 = hit[:2 * ho, :2 * wo].view(ho, 2, wo, 2, c)
            g = d4[i].float()
            for k in range(4):
                m = i4[i] == k
                a6[:, k >> 1, :, k & 1] = torch.where(m, g, 0.0)
                h6[:, k >> 1, :, k & 1] = m
            exp = torch.where(hit, (b + add).to(T), pre[i])
            self._exact(lab, after[i] == exp)

    def _chk_pool_bnsums(self, dt, dyp, idx, r, mean, inv, part):
        n, h, w, c = r.n, r.h, r.w, r.c
        ho, wo = h // 2, w // 2
        lab = f"pool_bnsums {n}x{h}x{w}x{c}"
        rt, d4, i4 = r.tensor(), dyp.view(n, ho, wo, c), idx.view(n, ho, wo, c)
        mu, iv = mean.to(F64), inv.to(F64)
        s = torch.zeros(2, c, dtype=F64, device=part.device)
        sa = torch.zeros_like(s)
        for i in range(n):
            win = rt[i, :2 * ho, :2 * wo].to(F64).view(ho, 2, wo, 2, c).permute(0, 2, 1, 3, 4).reshape(ho, wo, 4, c)
            rv = win.gather(2, i4[i].long().unsqueeze(2)).squeeze(2)
            g = d4[i].to(F64)
            t = g * (rv - mu) * iv
            s[0] += g.sum((0, 1))
            s[1] += t.sum((0, 1))
            sa[0] += g.abs().sum((0, 1))
            sa[1] += t.abs().sum((0, 1))
        tot = part.view(-1, 2, c).to(F64).sum(0)
        self._sums(lab, tot, s, sa)

    def _chk_pool_of_stored(self, lab, dt, y, pool_out, pool_idx, pool_sign):
        """The 2x2 pooling fused into a conv epilogue (cnnitmo_conv3x3_fwd_pool), bit-exact on
        the STORED output y: per channel the first maximum of sign(pool_sign) * y in window
        order (pool_sign None: of y; sign 0: the first element), the value stored there and
        its window index."""
        n, h, w, c = y.n, y.h, y.w, y.c
        ho, wo = h // 2, w // 2
        yt = y.tensor()
        p4, i4 = pool_out.view(n, ho, wo, c), pool_idx.view(n, ho, wo, c)
        m = torch.ones(c, dtype=F64, device=yt.device) if pool_sign is None else torch.sign(pool_sign.to(F64))
        for i in range(n):
            win = yt[i].to(F64).view(ho, 2, wo, 2, c).permute(0, 2, 1, 3, 4).reshape(ho, wo, 4, c)
            key = win * m
            first = (key == key.max(2).values.unsqueeze(2)).to(torch.uint8).argmax(2)
            self._exact(lab + " pool idx", i4[i].long() == first)
            self._exact(lab + " pool value", p4[i].to(F64) == win.gather(2, first.unsqueeze(2)).squeeze(2))

    def _chk_pool_bnsums_pooled(self, dt, dyp, pr, n, h, w, c, mean, inv, part):
        ho, wo = h // 2, w // 2
        lab = f"pool_bnsums_pooled {n}x{h}x{w}x{c}"
        d4, p4 = dyp.view(n, ho, wo, c), pr.view(n, ho, wo, c)
        mu, iv = mean.to(F64), inv.to(F64)
        s = torch.zeros(2, c, dtype=F64, device=part.device)
        sa = torch.zeros_like(s)
        for i in range(n):
            g = d4[i].to(F64)
            t = g * (p4[i].to(F64) - mu) * iv
            s[0] += g.sum((0, 1))
            s[1] += t.sum((0, 1))
            sa[0] += g.abs().sum((0, 1))
            sa[1] += t.abs().sum((0, 1))
        self._sums(lab, part.view(-1, 2, c).to(F64).sum(0), s, sa)

    # ---- BatchNormalization forward -------------------------------------------------
    def _pre_bn_fwd_finalize(self, stats, rows, c, groups, count, gamma, beta, mmean, mvar, *a, **k):
        return None if mmean is None else (mmean.clone(), mvar.clone())

    def _chk_bn_fwd_finalize(self, stats, rows, c, groups, count, gamma, beta, mmean, mvar, momentum, eps,
                             scale, shift, smean, sinv, pre=None):
        lab = f"bn_fwd_finalize c={c} groups={groups} count={int(count)}"
        st = stats.view(rows, 2, groups, c).to(F64)
        s1, s2 = st[:, 0].sum((0, 1)), st[:, 1].sum((0, 1))
        a1, a2 = st[:, 0].abs().sum((0, 1)), st[:, 1].abs().sum((0, 1))
        cnt = float(count)
        mean = s1 / cnt
        var = (s2 / cnt - mean * mean).clamp_min(0.0)
        e32, m32 = _f32(eps), _f32(momentum)
        inv = 1.0 / torch.sqrt(var + e32)
        g, b = gamma.to(F64), beta.to(F64)
        sc = g * inv
        # fp64 summation-order noise of the stat totals, propagated (tiny next to fp32 rounding)
        nz = 1e-14 * (a1 / cnt + a2 / cnt)
        self._close(lab + " mean", smean, mean, 2 * U32 * mean.abs() + 1e-14 * a1 / cnt + 1e-30)
        self._close(lab + " invstd", sinv, inv, 2 * U32 * inv + inv ** 3 * nz)
        self._close(lab + " scale", scale, sc, 2 * U32 * sc.abs() + (g * inv ** 3 * nz).abs() + 1e-30)
        self._close(lab + " shift", shift, b - mean * sc, 2 * U32 * (b.abs() + (mean * sc).abs()) + 1e-30)
        if mmean is not None:
            mm0, mv0 = pre
            var_u = var * (cnt / (cnt - 1.0)) * (cnt / (cnt - (1.0 + e32)))
            mmr = mm0.to(F64) * m32 + mean * (1.0 - m32)
            mvr = mv0.to(F64) * m32 + var_u * (1.0 - m32)
            self._close(lab + " moving_mean", mmean, mmr, 2 * U32 * (mm0.to(F64).abs() + mean.abs()) + 1e-30)
            self._close(lab + " moving_var (Bessel n/(n-1) * n/(n-1-eps))", mvar, mvr,
                        2 * U32 * (mv0.to(F64).abs() + var_u) + nz + 1e-30)

    def _chk_bn_infer_coeffs(self, c, gamma, beta, mmean, mvar, eps, scale, shift):
        lab = f"bn_infer_coeffs c={c}"
        sc = gamma.to(F64) / torch.sqrt(mvar.to(F64) + _f32(eps))
        self._close(lab + " scale", scale, sc, 4 * U32 * sc.abs() + 1e-30)
        mm = mmean.to(F64)
        self._close(lab + " shift", shift, beta.to(F64) - mm * sc,
                    4 * U32 * (beta.to(F64).abs() + (mm * sc).abs()) + 1e-30)

    def _chk_bn_apply(self, dt, r, p, c, scale, shift, y, flags=0, seed=0, layer=0):
        drop = bool(flags & L.DROPOUT)
        lab = f"bn_apply p={p} c={c}" + (" + Dropout(0.5)" if drop else "")
        n = y.n
        yt = y.tensor().reshape(n, -1, c)
        r2 = r.view(p, c)
        s, h = scale.to(F64), shift.to(F64)
        acc = self._acc(lab, dt)
        hw = p // n
        col = torch.arange(c, device=r.device, dtype=torch.int64)
        for i in range(n):
            rv = self._img(r2, i, n).to(F64)
            ref = rv * s + h
            ext = 4 * U32 * ((rv * s).abs() + h.abs())
            got = yt[i]
            if drop:
                pix = torch.arange(i * hw, (i + 1) * hw, device=r.device, dtype=torch.int64)
                keep = dropout_keep(seed, layer, pix[:, None] * c + col[None, :])
                ref = torch.where(keep, 2.0 * ref, torch.zeros_like(ref))
                ext = torch.where(keep, 2.0 * ext, torch.zeros_like(ext))
                self._exact(lab + " dropped elements are 0", (got == 0) | keep)
            acc.add(got, ref, ext)
        acc.done()

    # ---- BatchNormalization backward ------------------------------------------------
    def _dy_img(self, dy, i, c, drop, seed, layer):
        """dy' of image i: the stored gradient (x2 / 0 under the Dropout mask), fp64 [hw][c]."""
        g = dy.tensor()[i].reshape(-1, c).to(F64)
        if drop:
            hw = g.shape[0]
            pix = torch.arange(i * hw, (i + 1) * hw, device=g.device, dtype=torch.int64)
            col = torch.arange(c, device=g.device, dtype=torch.int64)
            keep = dropout_keep(seed, layer, pix[:, None] * c + col[None, :])
            g = torch.where(keep, 2.0 * g, torch.zeros_like(g))
        return g

    def _r_img(self, r, i, n, h, w, c):
        rt = r.tensor() if hasattr(r, "tensor") else r.view(n, h, w, c)
        return rt[i].reshape(-1, c).to(F64)

    def _chk_bn_bwd_reduce(self, dt, dy, r, c, mean, inv, flags, seed, layer, part):
        drop = bool(flags & L.DROPOUT)
        n, h, w = dy.n, dy.h, dy.w
        lab = f"bn_bwd_reduce {n}x{h}x{w}x{c}" + (" (Dropout)" if drop else "")
        mu, iv = mean.to(F64), inv.to(F64)
        s = torch.zeros(2, c, dtype=F64, device=part.device)
        sa = torch.zeros_like(s)
        for i in range(n):
            g = self._dy_img(dy, i, c, drop, seed, layer)
            t = g * (self._r_img(r, i, n, h, w, c) - mu) * iv
            s[0] += g.sum(0)
            s[1] += t.sum(0)
            sa[0] += g.abs().sum(0)
            sa[1] += t.abs().sum(0)
        self._sums(lab, part.view(-1, 2, c).to(F64).sum(0), s, sa)

    def _chk_bn_bwd_finalize(self, part, rows, c, count, gamma, mean, inv, dgamma, dbeta, coef):
        lab = f"bn_bwd_finalize c={c} count={int(count)}"
        pt = part.view(rows, 2, c).to(F64)
        sdy, sdyr = pt[:, 0].sum(0), pt[:, 1].sum(0)
        ady, adyr = pt[:, 0].abs().sum(0), pt[:, 1].abs().sum(0)
        nz0, nz1 = 1e-14 * ady, 1e-14 * adyr
        if dgamma is not None:
            self._close(lab + " dgamma", dgamma, sdyr, 2 * U32 * sdyr.abs() + nz1 + 1e-30)
        if dbeta is not None:
            self._close(lab + " dbeta", dbeta, sdy, 2 * U32 * sdy.abs() + nz0 + 1e-30)
        cnt = float(count)
        iv, mu = inv.to(F64), mean.to(F64)
        a = gamma.to(F64) * iv
        b = a * iv * sdyr / cnt
        e = b * mu - a * sdy / cnt
        cf = coef.view(3, c)
        self._close(lab + " a", cf[0], a, 2 * U32 * a.abs() + 1e-30)
        self._close(lab + " b", cf[1], b, 4 * U32 * b.abs() + (a * iv * nz1 / cnt).abs() + 1e-30)
        self._close(lab + " e", cf[2], e, 4 * U32 * ((b * mu).abs() + (a * sdy / cnt).abs())
                    + (a * iv * nz1 / cnt * mu).abs() + (a * nz0 / cnt).abs() + 1e-30)

    def _bnb_apply_check(self, lab, dt, n, h, w, c, gfun, r, coef, nobn, dz, part, npar, gslack=None):
        """dz = [r>0]*(a*g - b*r + e) (or [r>0]*g) per image, g = gfun(i) fp64 [hw][c]; the
        bias-gradient partials (split by pixel parity when npar == 4) from the stored dz."""
        acc = self._acc(lab, dt)
        if not nobn:
            a, b, e = coef.view(3, c).to(F64)
        z2 = dz.view(n, h * w, c)
        ps = torch.zeros(npar, c, dtype=F64, device=dz.device)
        pa = torch.zeros_like(ps)
        for i in range(n):
            g = gfun(i)
            rv = self._r_img(r, i, n, h, w, c)
            if nobn:
                ref, ext = torch.where(rv > 0, g, torch.zeros_like(g)), None
            else:
                ref = torch.where(rv > 0, a * g - b * rv + e, torch.zeros_like(g))
                gs = g.abs() if gslack is None else gslack(i)
                ext = torch.where(rv > 0, 4 * U32 * (a.abs() * gs + (b * rv).abs() + e.abs()), torch.zeros_like(g))
            acc.add(z2[i], ref, ext)
            zs = z2[i].to(F64).view(h, w, c)
            if npar == 4:
                for ph in range(2):
                    for pw in range(2):
                        v = zs[ph::2, pw::2]
                        ps[ph * 2 + pw] += v.sum((0, 1))
                        pa[ph * 2 + pw] += v.abs().sum((0, 1))
            else:
                ps[0] += zs.sum((0, 1))
                pa[0] += zs.abs().sum((0, 1))
        acc.done()
        self._sums(lab + " db partials", part.view(-1, npar, c).to(F64).sum(0), ps, pa)

    def _chk_bn_bwd_apply(self, dt, dy, r, c, coef, flags, seed, layer, dz, part):
        drop, nobn, par = bool(flags & L.DROPOUT), bool(flags & L.NO_BN), bool(flags & L.PARITY)
        n, h, w = dy.n, dy.h, dy.w
        lab = (f"bn_bwd_apply {n}x{h}x{w}x{c}" + (" (Dropout)" if drop else "") + (" (parity)" if par else "")
               + (" (no BN)" if nobn else ""))
        self._bnb_apply_check(lab, dt, n, h, w, c, lambda i: self._dy_img(dy, i, c, drop, seed, layer), r, coef,
                              nobn, dz, part, 4 if par else 1)

    def _chk_bn_bwd_apply_pooled(self, dt, dy, r, c, coef, dyp, idx, dz, part):
        n, h, w = dy.n, dy.h, dy.w
        ho, wo = h // 2, w // 2
        lab = f"bn_bwd_apply_pooled {n}x{h}x{w}x{c}"
        d4, i4 = dyp.view(n, ho, wo, c), idx.view(n, ho, wo, c)

        def g(i, absval=False):
            t = dy.tensor()[i].to(F64)
            t = t.abs() if absval else t.clone()
            t6 = t[:2 * ho, :2 * wo].view(ho, 2, wo, 2, c)
            gp = d4[i].to(F64)
            gp = gp.abs() if absval else gp
            for k in range(4):
                t6[:, k >> 1, :, k & 1] += torch.where(i4[i] == k, gp, torch.zeros_like(gp))
            return t.reshape(-1, c)

        self._bnb_apply_check(lab, dt, n, h, w, c, g, r, coef, False, dz, part, 1, gslack=lambda i: g(i, True))

    def _chk_bn_bwd_apply_g3(self, dt, g3, wh, r, c, p, coef, dz, part):
        n = r.n if hasattr(r, "n") else 1
        h, w = (r.h, r.w) if hasattr(r, "h") else (p, 1)
        lab = f"bn_bwd_apply_g3 {n}x{h}x{w}x{c}"
        W3 = wh.view(3, c).to(F64)
        q = g3.view(n, h * w, 3)
        self._bnb_apply_check(lab, dt, n, h, w, c, lambda i: q[i].to(F64) @ W3, r, coef, False, dz, part, 1,
                              gslack=lambda i: q[i].to(F64).abs() @ W3.abs())

    def _chk_bn_consumer_sums(self, mode, w, raw, cout, cin_tot, ci0, c, db, vtab, mean, inv, part):
        lab = f"bn_consumer_sums mode {mode} cout={cout} cin={cin_tot} [{ci0},{ci0 + c})"
        taps = {1: 9, 2: 4, 3: 1}[mode]
        K = cout * taps
        W = w.view(K, cin_tot)[:, ci0:ci0 + c].to(F64)
        R = raw.view(K, cin_tot)[:, ci0:ci0 + c].to(F64)
        if mode == 1:
            bs = vtab.view(8, cout).to(F64)
            V = db.to(F64)[:, None].repeat(1, 9)
            for t in range(9):
                rr, qq = t // 3, t % 3
                o = torch.zeros(cout, dtype=F64, device=w.device)
                if rr == 0:
                    o += bs[0]
                if rr == 2:
                    o += bs[1]
                if qq == 0:
                    o += bs[2]
                if qq == 2:
                    o += bs[3]
                if rr == 0 and qq == 0:
                    o -= bs[4]
                if rr == 0 and qq == 2:
                    o -= bs[5]
                if rr == 2 and qq == 0:
                    o -= bs[6]
                if rr == 2 and qq == 2:
                    o -= bs[7]
                V[:, t] -= o
            V = V.reshape(K)
        elif mode == 2:
            V = vtab.view(K).to(F64)
        else:
            V = db.view(K).to(F64)
        mu, iv = mean.to(F64), inv.to(F64)
        rows = L.CONSUMER_ROWS
        pr = part.view(rows, 2, c).to(F64)
        for rr in range(rows):  # each grid row sums its own contiguous (co, tap) range
            k0, k1 = (K * rr) // rows, (K * (rr + 1)) // rows
            wv = (W[k0:k1] * V[k0:k1, None])
            wr = W[k0:k1] * R[k0:k1]
            swv, swr = wv.sum(0), wr.sum(0)
            nz = 1e-13 * (wv.abs().sum(0) + wr.abs().sum(0))
            self._close(lab + f" row {rr} sum dy", pr[rr, 0], swv, 2 * U32 * swv.abs() + nz + 1e-30)
            t1 = iv * (swr - mu * swv)
            self._close(lab + f" row {rr} sum dy*rhat", pr[rr, 1], t1,
                        2 * U32 * t1.abs() + iv * (nz * (1 + mu.abs())) + 1e-30)

    def _chk_colsum(self, part, rows, cols, groups, out):
        lab = f"colsum rows={rows} cols={cols} groups={groups}"
        pt = part.view(rows, groups, cols // groups).to(F64)
        ref = pt.sum((0, 1))
        self._close(lab, out, ref, 2 * U32 * ref.abs() + 1e-13 * pt.abs().sum((0, 1)) + 1e-30)

    def _chk_border_sums(self, dt, dz, n, h, w, c, part):
        lab = f"border_sums {n}x{h}x{w}x{c}"
        d4 = dz.view(n, h, w, c)
        s = torch.zeros(8, c, dtype=F64, device=dz.device)
        sa = torch.zeros_like(s)
        for i in range(n):
            v = d4[i].to(F64)
            terms = [v[0], v[h - 1], v[:, 0], v[:, w - 1], v[0, 0][None], v[0, w - 1][None], v[h - 1, 0][None],
                     v[h - 1, w - 1][None]]
            for k, t in enumerate(terms):
                s[k] += t.sum(0)
                sa[k] += t.abs().sum(0)
        self._sums(lab, part.view(-1, 8, c).to(F64).sum(0), s, sa)

    # ---- head: Conv2D(3, 1, sigmoid) + MSE + accuracy ---------------------------------
    def _head_ref(self, x, i, h_valid, wt, b, aff):
        """(yhat, z slack, x image) of image i in fp64; yhat [h, w, 3] over all rows."""
        cin = x.c
        xi = x.tensor()[i].to(F64)
        W = wt.view(3, cin).to(F64)
        y_in = xi * aff[0].to(F64) + aff[1].to(F64) if aff is not None else xi
        z = y_in @ W.t() + b.to(F64)
        # fp32 evaluation: folded weights/bias, the 3 dot products over cin channels
        dz = 16 * U32 * ((xi.abs() * (aff[0].to(F64).abs() if aff is not None else 1.0)) @ W.abs().t()
                        + (aff[1].to(F64).abs() @ W.abs().t() if aff is not None else 0.0) + b.to(F64).abs())
        return torch.sigmoid(z), dz, xi

    def _chk_head_fwd(self, dt, x, h_valid, wt, b, yhat, aff=None):
        n = x.n
        lab = f"head_fwd {n}x{x.h}x{x.w}x{x.c} (valid {h_valid})"
        yt = yhat.view(n, h_valid, x.w, 3)
        for i in range(n):
            yh, dzs, _ = self._head_ref(x, i, h_valid, wt, b, aff)
            yh, dzs = yh[:h_valid], dzs[:h_valid]
            self._close(lab, yt[i], yh, 0.25 * dzs + 1e-6 * yh + 1e-7)

    def _head_bwd(self, lab, dt, x, h_valid, wt, b, target, part, aff, g3=None, dx=None, grad_numel=0.0):
        n, h, w, cin = x.n, x.h, x.w, x.c
        numel = float(grad_numel) if grad_numel and grad_numel > 0 else float(n * h_valid * w * 3)
        inv_n = _f32(1.0 / numel)
        tt = target.view(n, h_valid, w, 3)
        loss = corr = 0.0
        amb = 0
        db = torch.zeros(3, dtype=F64, device=wt.device)
        dbb, dba = torch.zeros_like(db), torch.zeros_like(db)
        dW = torch.zeros(3, cin, dtype=F64, device=wt.device)
        dWb, dWa = torch.zeros_like(dW), torch.zeros_like(dW)
        lsl = 0.0
        accx = self._acc(lab + " dx", dt) if dx is not None else None
        g3v = g3.view(n, h, w, 3) if g3 is not None else None
        W = wt.view(3, cin).to(F64)
        for i in range(n):
            yh, dzs, xi = self._head_ref(x, i, h_valid, wt, b, aff)
            t = tt[i].to(F64)
            yv = yh[:h_valid]
            e = yv - t
            dyh = 0.25 * dzs[:h_valid] + 1e-6  # |fp32 yhat - exact| (dot products, expf, divide)
            loss += float((e * e).sum())
            lsl += float((2 * e.abs() * dyh + dyh * dyh).sum())
            at = t.argmax(2)  # first maximum (strict '>' scan in the kernel)
            ap = yv.argmax(2)
            corr += float((at == ap).sum())
            srt = yv.sort(2, descending=True).values
            amb += int(((srt[..., 0] - srt[..., 1]) <= 2 * dyh.amax(2)).sum())
            d = torch.zeros(h, w, 3, dtype=F64, device=wt.device)
            d[:h_valid] = 2.0 * e * yv * (1.0 - yv) * inv_n
            bd = torch.zeros_like(d)
            bd[:h_valid] = 2.0 * inv_n * (dyh * (0.25 + e.abs()) * 1.5) + 4 * U32 * d[:h_valid].abs()
            if g3v is not None:
                self._close(lab + " g3", g3v[i], d, bd + 1e-30)
            if dx is not None:
                accx.add(dx.view(n, h, w, cin)[i], d @ W, 4 * U32 * (d.abs() @ W.abs()) + bd @ W.abs())
            d2, bd2, x2 = d.reshape(-1, 3), bd.reshape(-1, 3), xi.reshape(-1, cin)
            db += d2.sum(0)
            dba += d2.abs().sum(0)
            dbb += bd2.sum(0)
            dW += d2.t() @ x2
            dWa += d2.abs().t() @ x2.abs()
            dWb += bd2.t() @ x2.abs()
        if accx is not None:
            accx.done()
        tot = part.view(-1, 5 + 3 * cin).to(F64).sum(0)
        self._close(lab + " loss sum", tot[0:1], torch.tensor([loss], dtype=F64, device=tot.device),
                    torch.tensor([1e-5 * loss + lsl], dtype=F64, device=tot.device))
        cerr = abs(float(tot[1]) - corr)
        self.log.append((lab + " correct count", "|got-ref| - near ties", cerr - amb))
        assert cerr <= amb, f"{lab}: correct count {float(tot[1])} vs {corr} (only {amb} near ties)"
        self._close(lab + " db", tot[2:5], db, 1e-5 * dba + dbb + 1e-30)
        self._close(lab + " dW (raw)", tot[5:].view(3, cin), dW, 1e-5 * dWa + dWb + 1e-30)

    def _chk_head_fwd_bwd_g3(self, dt, x, h_valid, wt, b, target, g3, part, aff=None, grad_numel=0.0):
        lab = f"head_fwd_bwd_g3 {x.n}x{x.h}x{x.w}x{x.c} (valid {h_valid})" + (" (folded BN)" if aff else "")
        self._head_bwd(lab, dt, x, h_valid, wt, b, target, part, aff, g3=g3, grad_numel=grad_numel)

    def _chk_head_fwd_bwd(self, dt, x, h_valid, wt, b, target, dx, part, aff=None, grad_numel=0.0):
        lab = f"head_fwd_bwd {x.n}x{x.h}x{x.w}x{x.c} (valid {h_valid})" + (" (folded BN)" if aff else "")
        self._head_bwd(lab, dt, x, h_valid, wt, b, target, part, aff, dx=dx, grad_numel=grad_numel)

    def _chk_head_finalize(self, part, rows, cin, numel, loss_acc, dw, db, aff=None, raw=None):
        lab = f"head_finalize cin={cin} numel={int(numel)}"
        pt = part.view(rows, 5 + 3 * cin).to(F64)
        s, sa = pt.sum(0), pt.abs().sum(0)
        nz = 1e-13 * sa
        nm = float(numel)
        ref = torch.stack([s[0] / nm, s[1] / (nm / 3.0)])
        self._close(lab + " loss, acc", loss_acc, ref, 2 * U32 * ref.abs() + torch.stack([nz[0] / nm, nz[1]]) + 1e-30)
        self._close(lab + " db", db, s[2:5], 2 * U32 * s[2:5].abs() + nz[2:5] + 1e-30)
        sw = s[5:].view(3, cin)
        if aff is not None:
            fs, fh = aff[0].to(F64), aff[1].to(F64)
            ref = sw * fs + s[2:5, None] * fh
            bnd = 2 * U32 * ((sw * fs).abs() + (s[2:5, None] * fh).abs()) + nz[5:].view(3, cin) * fs.abs() \
                + nz[2:5, None] * fh.abs()
        else:
            ref, bnd = sw, 2 * U32 * sw.abs() + nz[5:].view(3, cin)
        self._close(lab + " dW" + (" (folded)" if aff is not None else ""), dw.view(3, cin), ref, bnd + 1e-30)
        if raw is not None:
            self._close(lab + " raw dW", raw.view(3, cin), sw, 2 * U32 * sw.abs() + nz[5:].view(3, cin) + 1e-30)

    # ---- RMSprop ------------------------------------------------------------------------
    def _pre_rmsprop(self, p, g, a, *args, **kw):
        return p.clone(), a.clone()

    def _chk_rmsprop(self, p, g, a, lr, rho, eps, grad_scale=1.0, pre=None):
        lab = f"rmsprop n={p.numel()}"
        p0, a0 = (t.to(F64) for t in pre)
        lr, rho, eps, gs = _f32(lr), _f32(rho), _f32(eps), _f32(grad_scale)
        one_m = float(np.float32(1.0) - np.float32(rho))
        gr = g.to(F64) * gs
        a1 = rho * a0 + one_m * gr * gr
        stp = lr * gr / (torch.sqrt(a1) + eps)
        self._close(lab + " accumulator", a, a1, 4 * U32 * a1 + 1e-300)
        self._close(lab + " params", p, p0 - stp, 2 * U32 * p0.abs() + 8 * U32 * stp.abs() + 1e-300)

    # ---- weight preparation and BN folding (per step) -----------------------------------
    def _chk_prep_conv3x3(self, dt, w32, cout, cin, wf, wflip):
        lab = f"prep_conv3x3 {cout}x3x3x{cin}"
        T = _tdt(dt)
        ref = w32.view(cout, 3, 3, cin).to(T)
        self._exact(lab + " fwd", wf.view(cout, 3, 3, cin) == ref)
        if wflip is not None:
            fl = ref.flip(1, 2).permute(3, 1, 2, 0)  # [cin][2-r][2-s][cout]
            self._exact(lab + " flipped", wflip.view(-1)[:cin * 9 * cout].view(cin, 3, 3, cout) == fl)

    def _chk_prep_tconv(self, dt, k32, cout, cin, kf, kT):
        lab = f"prep_tconv 2x2x{cout}x{cin}"
        ref = k32.view(4, cout, cin).to(_tdt(dt))
        self._exact(lab + " fwd", kf.view(4, cout, cin) == ref)
        self._exact(lab + " transposed", kT.view(cin, 4, cout) == ref.permute(2, 0, 1))

    def _chk_prep_c3(self, dt, w32, cout, wp):
        ref = torch.zeros(cout, 32, dtype=_tdt(dt), device=w32.device)
        ref[:, :27] = w32.view(cout, 27).to(_tdt(dt))
        self._exact(f"prep_c3 {cout}", wp.view(cout, 32) == ref)

    def _chk_fold_conv3x3(self, dt, w32, b, scale, shift, cout, cin, wout, bout, border):
        lab = f"fold_conv3x3 {cout}x3x3x{cin}"
        W = w32.view(cout, 9, cin)
        ws = W * scale if scale is not None else W
        self._exact(lab + " W*s", wout.view(cout, 9, cin) == ws.to(_tdt(dt)))
        Wd = W.to(F64)
        hd = shift.to(F64) if shift is not None else torch.zeros(cin, dtype=F64, device=W.device)
        u = Wd @ hd  # [cout][9]
        ua = Wd.abs() @ hd.abs()
        bd = b.to(F64) if b is not None else torch.zeros(cout, dtype=F64, device=W.device)
        # fp32 block-tree sums over cin (<= 11 levels) and the 9-tap sequential sum
        self._close(lab + " bias", bout, bd + u.sum(1), 32 * U32 * (bd.abs() + ua.sum(1)) + 1e-30)
        if border is not None:
            U = torch.stack([u[:, 0] + u[:, 1] + u[:, 2], u[:, 6] + u[:, 7] + u[:, 8], u[:, 0] + u[:, 3] + u[:, 6],
                             u[:, 2] + u[:, 5] + u[:, 8], u[:, 0], u[:, 2], u[:, 6], u[:, 8]], 1)
            Ua = torch.stack([ua[:, 0] + ua[:, 1] + ua[:, 2], ua[:, 6] + ua[:, 7] + ua[:, 8],
                              ua[:, 0] + ua[:, 3] + ua[:, 6], ua[:, 2] + ua[:, 5] + ua[:, 8], ua[:, 0], ua[:, 2],
                              ua[:, 6], ua[:, 8]], 1)
            self._close(lab + " border table", border.view(cout, 8), U, 32 * U32 * Ua + 1e-30)

    def _chk_fold_tconv(self, dt, k32, b, scale, shift, cout, cin, kout, bout):
        lab = f"fold_tconv 2x2x{cout}x{cin}"
        K = k32.view(4 * cout, cin)
        ks = K * scale if scale is not None else K
        self._exact(lab + " K*s", kout.view(4 * cout, cin) == ks.to(_tdt(dt)))
        hd = shift.to(F64) if shift is not None else torch.zeros(cin, dtype=F64, device=K.device)
        bd = (b.to(F64) if b is not None else torch.zeros(cout, dtype=F64, device=K.device)).repeat(4)
        self._close(lab + " bias", bout, bd + K.to(F64) @ hd,
                    32 * U32 * (bd.abs() + K.to(F64).abs() @ hd.abs()) + 1e-30)
