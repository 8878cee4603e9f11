"""Thin typed wrappers over the C ABI (include/cnn_itmo.h).

Activations are passed as ``View`` objects: an NHWC channel window
(buffer, ld, off) of a device buffer -- the zero-copy concatenation of
model.py:246-261 is just two views of one buffer.  torch supplies device
memory and the current HIP stream; every FLOP runs in libcnnitmo.so.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib as L
from ._lib import call, query

DTYPES = {"float32": (L.F32, torch.float32), "bfloat16": (L.BF16, torch.bfloat16)}


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


@dataclass
class View:
    """Element (p, c) of an [n, h, w, c] activation is buf[p*ld + off + c]."""
    buf: torch.Tensor
    n: int
    h: int
    w: int
    c: int
    ld: int
    off: int = 0

    @property
    def p(self):
        return self.n * self.h * self.w

    @property
    def ptr(self):
        return self.buf.data_ptr()

    def tensor(self):
        """[n, h, w, c] strided torch view (for tests / host copies)."""
        return self.buf.view(-1)[self.off:].as_strided((self.n, self.h, self.w, self.c),
                                                       (self.h * self.w * self.ld, self.w * self.ld, self.ld, 1))


def new_view(n, h, w, c, dtype, device="cuda"):
    return View(torch.empty(n * h * w * c, dtype=dtype, device=device), n, h, w, c, c, 0)


def workspace(nbytes, device="cuda"):
    return torch.empty(max(16, int(nbytes)), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------- convolutions
def conv3x3_fwd(dt, x: View, wt, bias, out: View, flags=0, aff=None, stats=None, border=None):
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_conv3x3_fwd", dt, x.ptr, x.ld, x.off, x.n, x.h, x.w, x.c, ptr(wt), ptr(bias),
         out.c, out.ptr, out.ld, out.off, flags, ptr(sc), ptr(sh), ptr(stats), ptr(border),
         stream_ptr())


def conv3x3_fwd_pool(dt, x: View, wt, bias, out: View, pool_out, pool_idx, pool_sign=None, flags=0, aff=None,
                     stats=None, border=None):
    """conv3x3_fwd + the output's 2x2 MaxPooling2D in the epilogue (cnnitmo_conv3x3_fwd_pool):
    pool_out / pool_idx [n, h/2, w/2, cout] dense; pool_sign [cout] (None: max)."""
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_conv3x3_fwd_pool", dt, x.ptr, x.ld, x.off, x.n, x.h, x.w, x.c, ptr(wt), ptr(bias),
         out.c, out.ptr, out.ld, out.off, flags, ptr(sc), ptr(sh), ptr(stats), ptr(border),
         ptr(pool_out), out.c, ptr(pool_idx), ptr(pool_sign), stream_ptr())


def pool_supported(dt, n, h, w, cin, cout):
    return query("cnnitmo_conv3x3_pool_supported", dt, n, h, w, cin, cout) == 1


def conv3x3_fwd_head(dt, x: View, wt, bias, cout, flags, aff, h_valid, head_w, head_b, yhat):
    """The inference forward of the last 3x3 ConvBN with the sigmoid head in its epilogue
    (cnnitmo_conv3x3_fwd_head): yhat [n, h_valid, w, 3] fp32; the conv output is not stored."""
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_conv3x3_fwd_head", dt, x.ptr, x.ld, x.off, x.n, x.h, x.w, x.c, ptr(wt), ptr(bias), cout, flags,
         ptr(sc), ptr(sh), h_valid, ptr(head_w), ptr(head_b), ptr(yhat), stream_ptr())


def head_supported(dt, n, h, w, cin, cout):
    return query("cnnitmo_conv3x3_head_supported", dt, n, h, w, cin, cout) == 1


def conv3x3_fwd_cat(dt, x1: View, x2: View, wt, bias, out: View, flags=0, aff=None, stats=None, border=None):
    """conv3x3_fwd over concatenate([x1, x2]) read from its members (cnnitmo_conv3x3_fwd_cat)."""
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_conv3x3_fwd_cat", dt, x1.ptr, x1.ld, x1.off, x1.c, x2.ptr, x2.ld, x2.off, x1.n, x1.h, x1.w,
         x1.c + x2.c, ptr(wt), ptr(bias), out.c, out.ptr, out.ld, out.off, flags, ptr(sc), ptr(sh), ptr(stats),
         ptr(border), stream_ptr())


def conv1tap_fwd(dt, cols, k, m, wt, bias, out: View, flags=0, aff=None, stats=None):
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_conv1tap_fwd", dt, ptr(cols), k, m, ptr(wt), ptr(bias), out.c, out.ptr, out.ld,
         out.off, flags, ptr(sc), ptr(sh), ptr(stats), stream_ptr())


def fwd_stat_rows(dt, m, ncols):
    return query("cnnitmo_fwd_stat_rows", dt, m, ncols)


def conv3x3_stat_rows(dt, n, h, w, cin, cout):
    return query("cnnitmo_conv3x3_stat_rows", dt, n, h, w, cin, cout)


def tconv_stat_rows(dt, n, h, w, cin, cout):
    """BN partial rows of tconv_fwd over an n x h x w input grid."""
    return query("cnnitmo_tconv2x2_stat_rows", dt, n, h, w, cin, cout)


def conv3x3_dgrad(dt, dz, n, h, w, cout, wflip, cin, dx: View):
    call("cnnitmo_conv3x3_dgrad", dt, ptr(dz), n, h, w, cout, ptr(wflip), cin, dx.ptr, dx.ld, dx.off,
         stream_ptr())


def conv3x3_dgrad_bn_rows(dt, n, h, w, cout, cin, c0, c1):
    return query("cnnitmo_conv3x3_dgrad_bn_rows", dt, n, h, w, cout, cin, c0, c1)


def conv3x3_dgrad_bn(dt, dz, n, h, w, cout, wflip, cin, dx, c0, c1, coef, r, dz_out, part, parity):
    """conv3x3_dgrad with the producer's BN backward fused (see cnn_itmo.h); dx: View or None."""
    rp, rld, roff = _rview(r, c1 - c0)
    call("cnnitmo_conv3x3_dgrad_bn", dt, ptr(dz), n, h, w, cout, ptr(wflip), cin,
         dx.ptr if dx is not None else None, dx.ld if dx is not None else cin, dx.off if dx is not None else 0,
         c0, c1, ptr(coef), rp, rld, roff, ptr(dz_out), ptr(part), 1 if parity else 0, stream_ptr())


def conv3x3_dgrad_bn_pooled_rows(dt, n, h, w, cout, cin):
    return query("cnnitmo_conv3x3_dgrad_bn_pooled_rows", dt, n, h, w, cout, cin)


def conv3x3_dgrad_bn_pooled(dt, dz, n, h, w, cout, wflip, cin, coef, r, dyp, idx, dz_out, part):
    """The skip member's input gradient + its MaxPooling2D gradient routed by idx, through the
    producer's BN backward (cnnitmo_conv3x3_dgrad_bn_pooled): the skip gradient is never stored."""
    rp, rld, roff = _rview(r, cin)
    call("cnnitmo_conv3x3_dgrad_bn_pooled", dt, ptr(dz), n, h, w, cout, ptr(wflip), cin, ptr(coef), rp, rld, roff,
         ptr(dyp), ptr(idx), ptr(dz_out), ptr(part), stream_ptr())


def tconv_dgrad_bn_rows(dt, n, h, w, cout, cin):
    return query("cnnitmo_tconv2x2_dgrad_bn_rows", dt, n, h, w, cout, cin)


def tconv_dgrad_bn(dt, dout, n, h, w, cout, kT, cin, coef, r, dz_out, part):
    """tconv2x2_dgrad with the producer's BN backward fused (see cnn_itmo.h)."""
    rp, rld, roff = _rview(r, cin)
    call("cnnitmo_tconv2x2_dgrad_bn", dt, ptr(dout), n, h, w, cout, ptr(kT), cin, ptr(coef), rp, rld, roff,
         ptr(dz_out), ptr(part), stream_ptr())


def conv_wgrad(dt, ntaps, x: View, dz, cout, dw, dw_cols=0, fold=None, raw=None):
    """fold = (scale, shift, db, border_sums) for a folded input BN, else None;
    raw (optional, dw-shaped fp32): the uncorrected dz (x) r sum."""
    nbytes = query("cnnitmo_wgrad_workspace_bytes", dt, x.n, x.h, x.w, x.c, cout, ntaps)
    ws = workspace(nbytes, dz.device)
    fs, fh, fdb, fb = fold if fold is not None else (None,) * 4
    call("cnnitmo_conv_wgrad", dt, ntaps, x.ptr, x.ld, x.off, ptr(dz), x.n, x.h, x.w, x.c, cout,
         ptr(dw), dw_cols, ptr(fs), ptr(fh), ptr(fdb), ptr(fb), ptr(raw), ws.data_ptr(), ws.numel(),
         stream_ptr())


def conv_wgrad_cat(dt, x1: View, x2: View, dz, cout, dw, fold=None, raw=None):
    """conv_wgrad (9 taps) over concatenate([x1, x2]) read from its members (cnnitmo_conv_wgrad_cat)."""
    cin = x1.c + x2.c
    ws = workspace(query("cnnitmo_wgrad_cat_workspace_bytes", x1.n, x1.h, x1.w, x1.c, cin, cout), dz.device)
    fs, fh, fdb, fb = fold if fold is not None else (None,) * 4
    call("cnnitmo_conv_wgrad_cat", dt, x1.ptr, x1.ld, x1.off, x1.c, x2.ptr, x2.ld, x2.off, ptr(dz), x1.n, x1.h,
         x1.w, cin, cout, ptr(dw), ptr(fs), ptr(fh), ptr(fdb), ptr(fb), ptr(raw), ws.data_ptr(), ws.numel(),
         stream_ptr())


def fwd_cat_supported(dt, n, h, w, c1, cin, cout):
    return query("cnnitmo_conv3x3_fwd_cat_supported", dt, n, h, w, c1, cin, cout) == 1


def wgrad_cat_supported(n, h, w, c1, cin, cout):
    return query("cnnitmo_wgrad_cat_workspace_bytes", n, h, w, c1, cin, cout) > 0


def conv_c3_stat_rows(n, h, w):
    return query("cnnitmo_conv_c3_stat_rows", n, h, w)


def conv_c3_fwd(dt, x, n, h_valid, h, w, wt, bias, out: View, flags=0, aff=None, stats=None):
    """First layer (bf16 or fp32 output), operands built from the fp32 input image (no
    im2col buffer)."""
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_conv_c3_fwd", dt, ptr(x), n, h_valid, h, w, ptr(wt), ptr(bias), out.ptr, out.ld, out.off, flags,
         ptr(sc), ptr(sh), ptr(stats), stream_ptr())


def conv_c3_wgrad(dt, x, n, h_valid, h, w, dz, dw):
    ws = workspace(query("cnnitmo_conv_c3_wgrad_workspace_bytes", n, h, w), dz.device)
    call("cnnitmo_conv_c3_wgrad", dt, ptr(x), n, h_valid, h, w, ptr(dz), ptr(dw), ws.data_ptr(), ws.numel(),
         stream_ptr())


def im2col_c3(dt, x, n, h_valid, h, w, cols):
    call("cnnitmo_im2col_c3", dt, ptr(x), n, h_valid, h, w, ptr(cols), stream_ptr())


def tconv_fwd(dt, x: View, k, bias, out: View, flags=0, aff=None, stats=None):
    assert x.ld == x.c and x.off == 0
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_tconv2x2_fwd", dt, x.ptr, x.n, x.h, x.w, x.c, ptr(k), ptr(bias), out.c, out.ptr,
         out.ld, out.off, flags, ptr(sc), ptr(sh), ptr(stats), stream_ptr())


def tconv_dgrad(dt, dout, n, h, w, cout, kT, cin, dx):
    call("cnnitmo_tconv2x2_dgrad", dt, ptr(dout), n, h, w, cout, ptr(kT), cin, ptr(dx), stream_ptr())


def tconv_wgrad(dt, x: View, dout, cout, dk, fold=None, raw=None):
    """fold = (scale, shift, parity_sums[4*cout]) for a folded input BN, else None."""
    assert x.ld == x.c and x.off == 0
    nbytes = query("cnnitmo_tconv2x2_wgrad_workspace_bytes", dt, x.n, x.h, x.w, x.c, cout)
    ws = workspace(nbytes, dout.device)
    fs, fh, fp = fold if fold is not None else (None,) * 3
    call("cnnitmo_tconv2x2_wgrad", dt, x.ptr, ptr(dout), x.n, x.h, x.w, x.c, cout, ptr(dk),
         ptr(fs), ptr(fh), ptr(fp), ptr(raw), ws.data_ptr(), ws.numel(), stream_ptr())


def prep_conv3x3(dt, w32, cout, cin, wf, wflip):
    call("cnnitmo_prep_conv3x3_weights", dt, ptr(w32), cout, cin, ptr(wf), ptr(wflip), stream_ptr())


def prep_tconv(dt, k32, cout, cin, kf, kT):
    call("cnnitmo_prep_tconv2x2_weights", dt, ptr(k32), cout, cin, ptr(kf), ptr(kT), stream_ptr())


def prep_c3(dt, w32, cout, wp):
    call("cnnitmo_prep_c3_weights", dt, ptr(w32), cout, ptr(wp), stream_ptr())


def fold_conv3x3(dt, w32, b, scale, shift, cout, cin, wout, bout, border):
    call("cnnitmo_fold_conv3x3", dt, ptr(w32), ptr(b), ptr(scale), ptr(shift), cout, cin, ptr(wout),
         ptr(bout), ptr(border), stream_ptr())


def fold_tconv(dt, k32, b, scale, shift, cout, cin, kout, bout):
    call("cnnitmo_fold_tconv2x2", dt, ptr(k32), ptr(b), ptr(scale), ptr(shift), cout, cin, ptr(kout),
         ptr(bout), stream_ptr())


def border_rows(n):
    return query("cnnitmo_border_rows", n)


def border_sums(dt, dz, n, h, w, c, part):
    call("cnnitmo_border_sums", dt, ptr(dz), n, h, w, c, ptr(part), stream_ptr())


# ---------------------------------------------------------------- pooling
def maxpool_fwd(dt, x: View, y, idx, aff=None):
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_maxpool2x2_fwd", dt, x.ptr, x.ld, x.off, x.n, x.h, x.w, x.c, ptr(y), ptr(idx),
         ptr(sc), ptr(sh), stream_ptr())


def maxpool_bwd(dt, dy, idx, dx: View):
    call("cnnitmo_maxpool2x2_bwd", dt, ptr(dy), ptr(idx), dx.n, dx.h, dx.w, dx.c, dx.ptr, dx.ld,
         dx.off, stream_ptr())


# ---------------------------------------------------------------- batch norm
def reduce_ws(rows, cols, device):
    return workspace(query("cnnitmo_reduce_workspace_bytes", rows, cols), device)


def bn_fwd_finalize(stats, rows, c, groups, count, gamma, beta, mmean, mvar, momentum, eps,
                    scale, shift, smean, sinv):
    ws = reduce_ws(rows, 2 * groups * c, stats.device)
    call("cnnitmo_bn_fwd_finalize", ptr(stats), rows, c, groups, float(count), ptr(gamma), ptr(beta),
         ptr(mmean), ptr(mvar), momentum, eps, ptr(scale), ptr(shift), ptr(smean), ptr(sinv),
         ws.data_ptr(), stream_ptr())


def bn_infer_coeffs(c, gamma, beta, mmean, mvar, eps, scale, shift):
    call("cnnitmo_bn_infer_coeffs", c, ptr(gamma), ptr(beta), ptr(mmean), ptr(mvar), eps, ptr(scale),
         ptr(shift), stream_ptr())


def bn_apply(dt, r, p, c, scale, shift, y: View, flags=0, seed=0, layer=0):
    call("cnnitmo_bn_apply", dt, ptr(r), p, c, ptr(scale), ptr(shift), y.ptr, y.ld, y.off, flags,
         seed, layer, stream_ptr())


def bn_bwd_rows(p, c):
    return query("cnnitmo_bn_bwd_rows", p, c)


def _rview(r, c):
    """(ptr, ld, off) of a saved post-ReLU tensor given as a View or a contiguous [p][c] tensor."""
    if isinstance(r, View):
        return r.ptr, r.ld, r.off
    return ptr(r), c, 0


def bn_bwd_reduce(dt, dy: View, r, c, mean, inv, flags, seed, layer, part):
    rp, rld, roff = _rview(r, c)
    call("cnnitmo_bn_bwd_reduce", dt, dy.ptr, dy.ld, dy.off, rp, rld, roff, dy.p, c, ptr(mean),
         ptr(inv), flags, seed, layer, ptr(part), stream_ptr())


def bn_bwd_finalize(part, rows, c, count, gamma, mean, inv, dgamma, dbeta, coef):
    ws = reduce_ws(rows, 2 * c, part.device)
    call("cnnitmo_bn_bwd_finalize", ptr(part), rows, c, float(count), ptr(gamma), ptr(mean), ptr(inv),
         ptr(dgamma), ptr(dbeta), ptr(coef), ws.data_ptr(), stream_ptr())


def bn_bwd_apply(dt, dy: View, r, c, coef, flags, seed, layer, dz, part):
    """flags & L.PARITY: part columns are [4][c] split by (h&1, w&1) of dy's pixel."""
    rp, rld, roff = _rview(r, c)
    call("cnnitmo_bn_bwd_apply", dt, dy.ptr, dy.ld, dy.off, rp, rld, roff, dy.p, c, ptr(coef), flags,
         seed, layer, dy.h, dy.w, ptr(dz), ptr(part), stream_ptr())


def bn_bwd_apply_pooled(dt, dy: View, r, c, coef, dyp, idx, dz, part):
    """bn_bwd_apply with a deferred MaxPooling2D backward folded in: dy += dyp routed by idx."""
    rp, rld, roff = _rview(r, c)
    call("cnnitmo_bn_bwd_apply_pooled", dt, dy.ptr, dy.ld, dy.off, rp, rld, roff, dy.n, dy.h, dy.w, c,
         ptr(coef), ptr(dyp), ptr(idx), ptr(dz), ptr(part), stream_ptr())


def colsum(part, rows, cols, groups, out):
    ws = reduce_ws(rows, cols, part.device)
    call("cnnitmo_colsum", ptr(part), rows, cols, groups, ptr(out), ws.data_ptr(), stream_ptr())


# ---------------------------------------------------------------- head / optimizer
def head_fwd(dt, x: View, h_valid, wt, b, yhat, aff=None):
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_head_fwd", dt, x.ptr, x.n, x.h, h_valid, x.w, x.c, ptr(wt), ptr(b), ptr(sc),
         ptr(sh), ptr(yhat), stream_ptr())


def head_fwd_bwd(dt, x: View, h_valid, wt, b, target, dx, part, aff=None, grad_numel=0.0):
    """grad_numel: the MSE gradient's normaliser (0: this batch's element count; see cnn_itmo.h)."""
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_head_fwd_bwd", dt, x.ptr, x.n, x.h, h_valid, x.w, x.c, ptr(wt), ptr(b), ptr(sc),
         ptr(sh), ptr(target), ptr(dx), ptr(part), float(grad_numel), stream_ptr())


def head_fwd_bwd_g3(dt, x: View, h_valid, wt, b, target, g3, part, aff=None, grad_numel=0.0):
    """head_fwd_bwd whose input gradient leaves as g3 [p][3] (dx = g3 . W)."""
    sc, sh = aff if aff is not None else (None, None)
    call("cnnitmo_head_fwd_bwd_g3", dt, x.ptr, x.n, x.h, h_valid, x.w, x.c, ptr(wt), ptr(b), ptr(sc),
         ptr(sh), ptr(target), ptr(g3), ptr(part), float(grad_numel), stream_ptr())


def bn_bwd_apply_g3(dt, g3, wh, r, c, p, coef, dz, part):
    rp, rld, roff = _rview(r, c)
    call("cnnitmo_bn_bwd_apply_g3", dt, ptr(g3), ptr(wh), rp, rld, roff, p, c, ptr(coef), ptr(dz), ptr(part),
         stream_ptr())


def head_rows(p):
    return query("cnnitmo_head_rows", p)


def head_finalize(part, rows, cin, numel, loss_acc, dw, db, aff=None, raw=None):
    sc, sh = aff if aff is not None else (None, None)
    ws = reduce_ws(rows, 5 + 3 * cin, part.device)
    call("cnnitmo_head_finalize", ptr(part), rows, cin, float(numel), ptr(sc), ptr(sh),
         ptr(loss_acc), ptr(dw), ptr(db), ptr(raw), ws.data_ptr(), stream_ptr())


def bn_consumer_sums(mode, w, raw, cout, cin_tot, ci0, c, db, vtab, mean, inv, part):
    """part[CONSUMER_ROWS][2][c] = (sum dy, sum dy*rhat) of a BN output from its consumer's weight
    gradient (mode 1 conv3x3, 2 tconv, 3 head); see cnn_itmo.h."""
    call("cnnitmo_bn_consumer_sums", mode, ptr(w), ptr(raw), cout, cin_tot, ci0, c, ptr(db), ptr(vtab),
         ptr(mean), ptr(inv), ptr(part), stream_ptr())


def pool_bnsums(dt, dyp, idx, r: View, mean, inv, part):
    """The MaxPooling2D share of a folded BN output's backward sums (rows =
    bn_bwd_rows(pooled pixels, c)); r is the pool input's view."""
    call("cnnitmo_pool_bnsums", dt, ptr(dyp), ptr(idx), r.n, r.h, r.w, r.c, r.ptr, r.ld, r.off, ptr(mean),
         ptr(inv), ptr(part), stream_ptr())


def pool_bnsums_pooled(dt, dyp, pr, n, h, w, c, mean, inv, part):
    """pool_bnsums when the producer pooled in its epilogue: pr = r at each window index
    [n, h/2, w/2, c] dense (h, w: the pool INPUT's size)."""
    call("cnnitmo_pool_bnsums_pooled", dt, ptr(dyp), ptr(pr), n, h, w, c, ptr(mean), ptr(inv), ptr(part),
         stream_ptr())


def rmsprop(p, g, a, lr, rho, eps, grad_scale=1.0):
    call("cnnitmo_rmsprop", ptr(p), ptr(g), ptr(a), p.numel(), lr, rho, eps, grad_scale, stream_ptr())


def augment_affine(src, mats, flips, scale, dst):
    """src [n,h,w,c] uint8/fp32 device tensor; mats [n,6] fp64 and flips [n] int32 device
    tensors; dst [n,h,w,c] fp32 (cnnitmo_augment_affine)."""
    n, h, w, c = src.shape
    assert src.is_contiguous() and dst.is_contiguous() and tuple(dst.shape) == (n, h, w, c)
    assert mats.dtype == torch.float64 and flips.dtype == torch.int32 and mats.numel() == 6 * n
    call("cnnitmo_augment_affine", 1 if src.dtype == torch.uint8 else 0, ptr(src), n, h, w, c, ptr(mats),
         ptr(flips), float(scale), ptr(dst), stream_ptr())
