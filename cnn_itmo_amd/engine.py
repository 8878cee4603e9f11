"""Graph compiler + executor: Keras layer graph -> fused HIP-kernel stages.

Fusion rules (what the reference's graph, /root/reference/model.py:195-278,
needs; anything else raises NotImplementedError at compile time):

  Conv2D(3,'same') [+Activation('relu') | activation='relu'] [+BatchNormalization] [+Dropout]
      -> BlockStage 'c3'   (conv epilogue: bias+ReLU+BN partial sums; BN-apply(+dropout)
                            writes straight into its consumer's buffer / concat slice)
  first Conv2D(3,'same') on the 3-channel Input -> BlockStage 'c3in' (im2col-packed 1-tap GEMM)
  Conv2DTranspose(2, strides=2) + ReLU + BN      -> BlockStage 't2' (pixel-scatter epilogue)
  MaxPooling2D(2)                                -> PoolStage
  concatenate([...])                             -> ConcatStage (zero-copy: inputs are placed
                                                    as channel slices of one buffer)
  final Conv2D(3, 1, activation='sigmoid')       -> HeadStage (sigmoid + MSE + accuracy + grads)

Training BN uses per-replica batch statistics (Keras semantics per process).

BN folding (training): a BN without Dropout never materialises its output
y = r*scale + shift.  The conv epilogue stores r = relu(conv) straight into
the output Value (or its concat slice), the finalize writes scale/shift into
the Value's per-channel coefficient buffer, and every consumer folds the
affine: convs/tconvs fold it into their weights and bias each step
(cnnitmo_fold_*, exact zero-padding border table), the pool and the head apply
it on load, and the consumer's weight gradient gets the exact correction
s*dW(r) + h*V (cnnitmo_conv_wgrad / tconv2x2_wgrad fold arguments).  This
removes one read+write of every activation per step.  Dropout outputs stay
materialised (identity coefficients).
Every parameter lives in one flat fp32 buffer laid out in REVERSE stage order,
so backward produces gradients front-to-back -- the order the data-parallel
bucketer (dist.py) all-reduces them in.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from . import _lib as L
from .layers import (Activation, BatchNormalization, Concatenate, Conv2D, Conv2DTranspose, Dropout,
                     InputLayer, MaxPooling2D)

ALIGN = 16  # floats


class Value:
    """A materialised activation [n, h, w, c] (optionally a channel slice of a concat)."""

    def __init__(self, name, shape):
        self.name = name
        self.h, self.w, self.c = shape
        self.place = None  # (concat Value, channel offset)
        self.members = []  # for concat values: placed member Values
        self.buf = None
        self.gbuf = None
        self.gsep = False  # gradient in a dense buffer of its own, not the concat owner's slice
        self.ginit = False
        self.needs_grad = True
        self.folded = False  # holds r; the true value is r*cs + ch (per channel)
        self.producer = None  # BlockStage writing this value
        self.sum_consumers = 0  # >0: BN-backward sums come from this many consumers (no reduce pass)
        self.fuse_into = None  # the single conv3x3 consumer whose dgrad applies this BN's backward
        self.bn_contrib = []  # per-step partial-sum tensors [rows][2][c] from the consumers
        self.pool_route = None  # (pooled gradient, argmax idx): a deferred MaxPooling2D backward
        self.grad_g3 = None  # (g3 [p][3], head weights [3][c]): the gradient as the head's rank-3 factor
        # a deferred skip-path input gradient (dz, n, h, w, cout, flipped weights, c) of the concat
        # consumer: computed inside this value's BN backward (cnnitmo_conv3x3_dgrad_bn_pooled)
        self.gdefer = None
        self.cs = None  # coefficient buffers of the owner (persist across steps)
        self.ch = None
        self.split = False  # concat whose members keep dense buffers of their own (Engine._plan_split_concats)
        self.coef_src = None  # a fused pool's output: folded with its input's BN coefficients

    def owner(self):
        return self.place[0] if self.place else self

    def _own_buffer(self):
        """A member of a split concat holds its activation in a buffer of its own."""
        return not self.place or self.place[0].split

    def view(self, n):
        if self.split:
            raise RuntimeError(f"{self.name}: a split concatenate has no single view (read its members)")
        if not self._own_buffer():
            cv, off = self.place
            return ops.View(cv.buf, n, self.h, self.w, self.c, cv.c, off)
        return ops.View(self.buf, n, self.h, self.w, self.c, self.c, 0)

    def gview(self, n):
        if self.place and not self.gsep:
            cv, off = self.place
            return ops.View(cv.gbuf, n, self.h, self.w, self.c, cv.c, off)
        return ops.View(self.gbuf, n, self.h, self.w, self.c, self.c, 0)

    def ensure(self, n, dtype, device):
        if self.split:
            return  # the members allocate their own
        o = self if self._own_buffer() else self.owner()
        if o.buf is None:
            o.buf = torch.empty(n * o.h * o.w * o.c, dtype=dtype, device=device)

    def ensure_grad(self, n, dtype, device, zero=False):
        o = self if self.gsep else self.owner()
        if o.gbuf is None:
            o.gbuf = (torch.zeros if zero else torch.empty)(n * o.h * o.w * o.c, dtype=dtype, device=device)
            if zero:
                o.mark_grad()

    def ensure_coef(self, device):
        if self.coef_src is not None:
            return self.coef_src.ensure_coef(device)
        o = self.owner()
        if o.cs is None:
            o.cs = torch.ones(o.c, device=device, dtype=torch.float32)
            o.ch = torch.zeros(o.c, device=device, dtype=torch.float32)

    def coef(self):
        """(scale, shift) [c] fp32 slices of the owner's coefficient buffers."""
        if self.coef_src is not None:
            return self.coef_src.coef()
        o = self.owner()
        off = self.place[1] if self.place else 0
        return o.cs[off:off + self.c], o.ch[off:off + self.c]

    def mark_grad(self):
        self.ginit = True
        for m in self.members:
            m.ginit = True

    def release(self):
        self.buf = None
        self.gbuf = None
        self.ginit = False
        self.bn_contrib = []
        self.pool_route = None
        self.grad_g3 = None
        self.gdefer = None


class Stage:
    params = ()  # [(key, shape)] trainable, in flat-buffer order
    buffers = ()  # [(key, shape)] non-trainable

    def bind(self, eng):
        self.eng = eng


class BlockStage(Stage):
    def __init__(self, kind, conv, relu, bn, drop, drop_id, vin, vout):
        self.kind, self.conv, self.relu, self.bn, self.drop = kind, conv, relu, bn, drop
        self.pool = None  # the PoolStage whose 2x2 max-pool this conv's epilogue computes (Engine._plan_pool_fusion)
        self.head_ran = False  # this forward computed the head (predict with a fused head)
        self.head = None  # the HeadStage this conv's inference epilogue computes (Engine._plan_head_fusion)
        self.drop_id = drop_id
        self.vin, self.vout = vin, vout
        self.cin = vin.c if kind != "c3in" else 3
        self.cout = conv.filters
        self.name = conv.name
        k = conv.name
        if kind == "t2":
            kshape = (2, 2, self.cout, self.cin)
        else:
            kshape = (self.cout, 3, 3, self.cin)
        self.params = [(k + "/kernel", kshape), (k + "/bias", (self.cout,))]
        self.buffers = []
        if bn is not None:
            b = bn.name
            self.params += [(b + "/gamma", (self.cout,)), (b + "/beta", (self.cout,))]
            self.buffers = [(b + "/moving_mean", (self.cout,)), (b + "/moving_variance", (self.cout,))]

    def bind(self, eng):
        super().bind(eng)
        T = eng.tdtype
        cout, cin = self.cout, self.cin
        dev = eng.device
        if self.kind == "c3":
            self.w_fwd = torch.empty(cout * 9 * cin, dtype=T, device=dev)
            self.w_bwd = torch.empty(cout * 9 * cin, dtype=T, device=dev)
        elif self.kind == "c3in":
            self.w_fwd = torch.empty(cout * 32, dtype=T, device=dev)
            self.w_bwd = None
        else:
            self.w_fwd = torch.empty(4 * cout * cin, dtype=T, device=dev)
            self.w_bwd = torch.empty(4 * cout * cin, dtype=T, device=dev)
        self.foldable = self.kind != "c3in" and self.vin.folded
        # first layer without im2col (32 filters; other widths: im2col + 1-tap GEMM):
        # both dtypes run conv_c3's forward and weight gradient, training and inference
        self.direct_ok = self.kind == "c3in" and cout == 32
        self.direct = self.direct_ok
        if self.foldable:  # per-step folded copies (training)
            f32 = torch.float32
            self.w_fold = torch.empty_like(self.w_fwd)
            self.b_fold = torch.empty((4 if self.kind == "t2" else 1) * cout, dtype=f32, device=dev)
            self.border = torch.empty(8 * cout, dtype=f32, device=dev) if self.kind == "c3" else None
        if self.vout.folded:
            self.vout.ensure_coef(dev)
        self.fold_active = False
        self.fused = None  # (dz, part, rows) when the consumer's dgrad applied this stage's BN backward

    def prep(self):
        e = self.eng
        w = e.p(self.conv.name + "/kernel")
        if self.kind == "c3":
            ops.prep_conv3x3(e.dt, w, self.cout, self.cin, self.w_fwd, self.w_bwd)
        elif self.kind == "c3in":
            ops.prep_c3(e.dt, w, self.cout, self.w_fwd)
        else:
            ops.prep_tconv(e.dt, w, self.cout, self.cin, self.w_fwd, self.w_bwd)

    def _conv(self, n, out_view, flags, aff=None, stats=None):
        e = self.eng
        bias = e.p(self.conv.name + "/bias")
        if self.fold_active:
            cs, ch = self.vin.coef()
            w32 = e.p(self.conv.name + "/kernel")
            if self.kind == "c3":
                ops.fold_conv3x3(e.dt, w32, bias, cs, ch, self.cout, self.cin, self.w_fold, self.b_fold,
                                 self.border)
                if self.vin.split:
                    a, b = self.vin.members
                    ops.conv3x3_fwd_cat(e.dt, a.view(n), b.view(n), self.w_fold, self.b_fold, out_view, flags, aff,
                                        stats, border=self.border)
                elif self.pool is not None:
                    ops.conv3x3_fwd_pool(e.dt, self.vin.view(n), self.w_fold, self.b_fold, out_view,
                                         *self._pool_bufs(n), flags=flags, aff=aff, stats=stats, border=self.border)
                else:
                    ops.conv3x3_fwd(e.dt, self.vin.view(n), self.w_fold, self.b_fold, out_view, flags, aff,
                                    stats, border=self.border)
            else:
                ops.fold_tconv(e.dt, w32, bias, cs, ch, self.cout, self.cin, self.w_fold, self.b_fold)
                ops.tconv_fwd(e.dt, self.vin.view(n), self.w_fold, self.b_fold, out_view,
                              flags | L.BIAS_PER_COL, aff, stats)
            return
        if self.kind == "c3" and self.vin.split:
            a, b = self.vin.members
            ops.conv3x3_fwd_cat(e.dt, a.view(n), b.view(n), self.w_fwd, bias, out_view, flags, aff, stats)
        elif self.kind == "c3" and self.pool is not None:
            ops.conv3x3_fwd_pool(e.dt, self.vin.view(n), self.w_fwd, bias, out_view, *self._pool_bufs(n), flags=flags,
                                 aff=aff, stats=stats)
        elif self.kind == "c3":
            ops.conv3x3_fwd(e.dt, self.vin.view(n), self.w_fwd, bias, out_view, flags, aff, stats)
        elif self.kind == "c3in" and self.direct:
            ops.conv_c3_fwd(e.dt, e.x_in, n, e.h_valid, self.vout.h, self.vout.w, self.w_fwd, bias, out_view, flags,
                            aff, stats)
        elif self.kind == "c3in":
            ops.conv1tap_fwd(e.dt, self.cols, 32, n * self.vout.h * self.vout.w, self.w_fwd, bias,
                             out_view, flags, aff, stats)
        else:
            ops.tconv_fwd(e.dt, self.vin.view(n), self.w_fwd, bias, out_view, flags, aff, stats)

    def _head_fits(self, n):
        """The fused head addresses yhat [n][h_valid][w][3] fp32 with 32-bit offsets
        (cnnitmo_conv3x3_fwd_head); a larger batch takes the unfused conv + head_fwd path,
        whose head kernel only needs fewer than 2^31 pixels (e.g. fp32 4K at the default
        Model.predict batch of 32)."""
        return n * self.eng.h_valid * self.vout.w * 12 < (1 << 31)

    def _conv_head(self, n):
        """predict(): this conv with the sigmoid head in its epilogue, straight into the
        prediction buffer (cnnitmo_conv3x3_fwd_head); the conv's own output is never stored."""
        e, bn, cout = self.eng, self.bn, self.cout
        sc = torch.empty(cout, device=e.device, dtype=torch.float32)
        sh = torch.empty(cout, device=e.device, dtype=torch.float32)
        ops.bn_infer_coeffs(cout, e.p(bn.name + "/gamma"), e.p(bn.name + "/beta"), e.b(bn.name + "/moving_mean"),
                            e.b(bn.name + "/moving_variance"), bn.epsilon, sc, sh)
        hd = self.head
        ops.conv3x3_fwd_head(e.dt, self.vin.view(n), self.w_fwd, e.p(self.conv.name + "/bias"), cout,
                             (L.RELU if self.relu else 0) | L.AFFINE, (sc, sh), e.h_valid, e.p(hd.name + "/kernel"),
                             e.p(hd.name + "/bias"), e._yhat)

    def _pool_bufs(self, n):
        """(pooled output, window indices, pool sign) for the fused MaxPooling2D: in training
        the epilogue stores r with the BN folded into the consumers, so it pools r by the
        sign of gamma (= the sign of the BN scale); in inference it stores y and pools by the
        maximum."""
        e, pv = self.eng, self.pool.vout
        pv.ensure(n, e.tdtype, e.device)
        self.pool.idx = torch.empty(n * pv.h * pv.w * pv.c, dtype=torch.uint8, device=e.device)
        sign = e.p(self.bn.name + "/gamma") if (e.training and self.vout.folded) else None
        return pv.buf, self.pool.idx, sign

    def _gemm_rows(self, n):
        if self.kind == "t2":
            return n * self.vin.h * self.vin.w, 4 * self.cout
        return n * self.vout.h * self.vout.w, self.cout

    def _sum_targets(self):
        """(value, channel offset) of this stage's inputs whose BN-backward sums it supplies."""
        if self.kind == "c3in":
            return []
        members = self.vin.members if self.vin.members else [self.vin]
        out = []
        for m in members:
            if m.sum_consumers:
                out.append((m, m.place[1] if m.place else 0))
        return out

    def forward(self, n, training):
        e = self.eng
        cout = self.cout
        P = n * self.vout.h * self.vout.w
        self.fold_active = training and self.foldable
        self.direct = self.direct_ok
        self.head_ran = False
        if not training and self.head is not None and e._yhat is not None and self._head_fits(n):
            self._conv_head(n)
            self.head_ran = True
            return
        if self.kind == "c3in" and not self.direct:
            self.cols = torch.empty(P * 32, dtype=e.tdtype, device=e.device)
            ops.im2col_c3(e.dt, e.x_in, n, e.h_valid, self.vout.h, self.vout.w, self.cols)
        self.vout.ensure(n, e.tdtype, e.device)
        out = self.vout.view(n)
        if self.bn is None:
            if self.vout.place:
                raise NotImplementedError("a ReLU-only conv whose output feeds a concatenate")
            self._conv(n, out, L.RELU if self.relu else 0)
            self.r = self.vout.buf
            return
        bn = self.bn
        g, b = e.p(bn.name + "/gamma"), e.p(bn.name + "/beta")
        mm, mv = e.b(bn.name + "/moving_mean"), e.b(bn.name + "/moving_variance")
        if not training:
            sc = torch.empty(cout, device=e.device, dtype=torch.float32)
            sh = torch.empty(cout, device=e.device, dtype=torch.float32)
            ops.bn_infer_coeffs(cout, g, b, mm, mv, bn.epsilon, sc, sh)
            self._conv(n, out, (L.RELU if self.relu else 0) | L.AFFINE, aff=(sc, sh))
            return
        m, ncols = self._gemm_rows(n)
        if self.kind == "c3":
            rows = ops.conv3x3_stat_rows(e.dt, n, self.vout.h, self.vout.w, self.cin, cout)
        elif self.kind == "t2":
            rows = ops.tconv_stat_rows(e.dt, n, self.vin.h, self.vin.w, self.cin, cout)
        elif self.direct:
            rows = ops.conv_c3_stat_rows(n, self.vout.h, self.vout.w)
        else:
            rows = ops.fwd_stat_rows(e.dt, m, ncols)
        stats = torch.empty(rows * 2 * ncols, device=e.device, dtype=torch.float32)
        if self.vout.folded:  # r goes straight into the output (slice); consumers fold the BN
            rview = out
        else:
            r = torch.empty(P * cout, dtype=e.tdtype, device=e.device)
            rview = ops.View(r, n, self.vout.h, self.vout.w, cout, cout, 0)
        self._conv(n, rview, (L.RELU if self.relu else 0) | L.STATS, stats=stats)
        if self.vout.folded:
            self.scale, self.shift = self.vout.coef()
        else:
            self.scale = torch.empty(cout, device=e.device, dtype=torch.float32)
            self.shift = torch.empty(cout, device=e.device, dtype=torch.float32)
        self.smean = torch.empty(cout, device=e.device, dtype=torch.float32)
        self.sinv = torch.empty(cout, device=e.device, dtype=torch.float32)
        ops.bn_fwd_finalize(stats, rows, cout, 4 if self.kind == "t2" else 1, P, g, b,
                            mm if e.update_moving else None, mv if e.update_moving else None,
                            bn.momentum, bn.epsilon, self.scale, self.shift, self.smean, self.sinv)
        if not self.vout.folded:
            flags = L.DROPOUT if self.drop is not None else 0
            ops.bn_apply(e.dt, r, P, cout, self.scale, self.shift, out, flags, e.drop_seed, self.drop_id)
        self.r = rview

    def bn_coef(self, n):
        """BN-backward coefficients [3][cout] (and dgamma/dbeta) from the consumer-derived
        sums alone, for a consumer that applies the BN backward in its dgrad store."""
        e = self.eng
        v = self.vout
        assert v.sum_consumers and len(v.bn_contrib) == v.sum_consumers
        part = torch.cat(v.bn_contrib)
        v.bn_contrib = []
        coef = torch.empty(3 * self.cout, device=e.device, dtype=torch.float32)
        ops.bn_bwd_finalize(part, part.numel() // (2 * self.cout), self.cout, n * v.h * v.w,
                            e.p(self.bn.name + "/gamma"), self.smean, self.sinv, e.g(self.bn.name + "/gamma"),
                            e.g(self.bn.name + "/beta"), coef)
        return coef

    def backward(self, n):
        e = self.eng
        cout = self.cout
        P = n * self.vout.h * self.vout.w
        par = self.fold_active and self.kind == "t2"  # tconv wgrad fold needs per-tap sums of dz
        if self.fused is not None:  # dz and its column partials came from the consumer's dgrad
            dz, part2, rows = self.fused
            self.fused = None
        else:
            dz, part2, rows = self._bn_backward(n, P, par)
        self._weight_and_input_grads(n, P, par, dz, part2, rows)

    def _bn_backward(self, n, P, par):
        e = self.eng
        cout = self.cout
        if not self.vout.ginit:
            raise RuntimeError(f"{self.name}: output gradient not initialised")
        g3 = self.vout.grad_g3
        dy = self.vout.gview(n) if g3 is None and self.vout.gdefer is None else None
        rows = ops.bn_bwd_rows(P, cout)
        dz = torch.empty(P * cout, dtype=e.tdtype, device=e.device)
        part2 = torch.empty(rows * (4 if par else 1) * cout, device=e.device, dtype=torch.float32)
        flags = (L.DROPOUT if self.drop is not None else 0) | (L.PARITY if par else 0)
        if self.bn is not None:
            bn = self.bn
            v = self.vout
            if v.sum_consumers and len(v.bn_contrib) == v.sum_consumers:
                # sums from the consumers' weight gradients (cnnitmo_bn_consumer_sums): no pass over dy
                part = torch.cat(v.bn_contrib)
                prow = part.numel() // (2 * cout)
            else:
                if v.pool_route is not None:  # route the deferred pool gradient before the reduce
                    ops.maxpool_bwd(e.dt, v.pool_route[0], v.pool_route[1], dy)
                    v.pool_route = None
                part = torch.empty(rows * 2 * cout, device=e.device, dtype=torch.float32)
                ops.bn_bwd_reduce(e.dt, dy, self.r, cout, self.smean, self.sinv, flags, e.drop_seed,
                                  self.drop_id, part)
                prow = rows
            v.bn_contrib = []
            coef = torch.empty(3 * cout, device=e.device, dtype=torch.float32)
            ops.bn_bwd_finalize(part, prow, cout, P, e.p(bn.name + "/gamma"), self.smean, self.sinv,
                                e.g(bn.name + "/gamma"), e.g(bn.name + "/beta"), coef)
            if g3 is not None:  # dy = g3 . W_head, formed inside the apply
                assert not flags and v.pool_route is None, "rank-3 head gradient with dropout/parity/pool"
                ops.bn_bwd_apply_g3(e.dt, g3[0], g3[1], self.r, cout, P, coef, dz, part2)
                v.grad_g3 = None
            elif v.pool_route is not None and v.gdefer is not None:
                # the concat consumer's skip-path dgrad, deferred to here: its gradient is never
                # stored, the pool's is routed in, the BN backward applied (one launch)
                assert not flags, "pool routing with dropout/parity"
                dzs, hs, ws, cz, wb = v.gdefer
                rows = ops.conv3x3_dgrad_bn_pooled_rows(e.dt, n, hs, ws, cz, cout)
                part2 = torch.empty(rows * cout, device=e.device, dtype=torch.float32)
                ops.conv3x3_dgrad_bn_pooled(e.dt, dzs, n, hs, ws, cz, wb, cout, coef, self.r, v.pool_route[0],
                                            v.pool_route[1], dz, part2)
                v.pool_route = None
                v.gdefer = None
            elif v.pool_route is not None:
                assert not flags, "pool routing with dropout/parity"
                ops.bn_bwd_apply_pooled(e.dt, dy, self.r, cout, coef, v.pool_route[0], v.pool_route[1], dz,
                                        part2)
                v.pool_route = None
            else:
                ops.bn_bwd_apply(e.dt, dy, self.r, cout, coef, flags, e.drop_seed, self.drop_id, dz, part2)
        else:
            ops.bn_bwd_apply(e.dt, dy, self.r, cout, None, flags | L.NO_BN, e.drop_seed,
                             self.drop_id, dz, part2)
        return dz, part2, rows

    def _fused_target(self, n, targets):
        """The (value, channel offset) among `targets` whose BN backward this stage's dgrad
        applies (cnnitmo_conv3x3_dgrad_bn), with its partial-sum row count; or None."""
        e = self.eng
        if self.kind not in ("c3", "t2") or not self.vin.needs_grad:
            return None
        for m, ci0 in targets:
            if m.fuse_into is self and m.sum_consumers == 1:
                if self.kind == "c3" and self._split_fused(ci0, m.c, n):
                    rows = ops.conv3x3_dgrad_bn_rows(e.dt, n, self.vout.h, self.vout.w, self.cout, m.c, 0, m.c)
                elif self.kind == "c3":
                    rows = ops.conv3x3_dgrad_bn_rows(e.dt, n, self.vout.h, self.vout.w, self.cout, self.cin, ci0,
                                                     ci0 + m.c)
                elif ci0 == 0 and m.c == self.cin and m.producer.kind != "t2":  # (no parity sums here)
                    rows = ops.tconv_dgrad_bn_rows(e.dt, n, self.vin.h, self.vin.w, self.cout, self.cin)
                else:
                    rows = 0
                if rows > 0:
                    return m, ci0, rows
        return None

    def _skip_member(self, ci0):
        """The concat member holding input channels [0, ci0) when it is exactly one value
        without a gradient yet (dec9's `conv1`, 64 B of every 192-B row): the split dgrad
        then writes its gradient to a dense buffer of its own.  Nothing reads that gradient
        through the concat."""
        ms = [v for v in self.vin.members if v.place and v.place[1] < ci0]
        if len(ms) == 1 and ms[0].place[1] == 0 and ms[0].c == ci0 and not ms[0].ginit:
            return ms[0]
        return None

    def _defer_skip(self, skip, n):
        """dec9's skip path (conv1, model.py:209-211 + 261): when conv1's only other reader is
        pool1 and its BN-backward sums come from its consumers, its input gradient is not
        launched here but inside conv1's BN backward, where pool1's gradient is routed in
        (cnnitmo_conv3x3_dgrad_bn_pooled): the 32-channel skip gradient is neither written
        nor read back, and the stand-alone pooled BN-backward apply disappears (otherwise: the
        separate dgrad + bn_bwd_apply_pooled).  (_split_fused splits dec7's and dec8's input
        gradients for the same purpose.)"""
        e = self.eng
        prod = skip.producer
        if prod is None or prod.bn is None or prod.drop is not None or not skip.folded or skip.sum_consumers != 2:
            return False
        pools = [s for s in e.stages if isinstance(s, PoolStage) and s.vin is skip]
        if len(pools) != 1 or prod.kind == "t2":
            return False
        return ops.conv3x3_dgrad_bn_pooled_rows(e.dt, n, self.vout.h, self.vout.w, self.cout, skip.c) > 0

    def _split_fused(self, ci0, c, n):
        """The input gradient of a concat consumer as two launches: the up columns [ci0, cin)
        as a dgrad with the fused BN backward, and the skip columns [0, ci0) apart.
        dec9 (concat [skip 32 | up 64], model.py:261): always -- one launch would need
        48-column blocks whose epilogue straddles both (measured 15 ms); its skip part is a
        plain dgrad, or deferred (_defer_skip).  dec7 / dec8 (model.py:251, 256): when the
        skip member's gradient is deferred into its producer's BN backward with its pool's
        route.  Otherwise: one launch."""
        if not (ci0 > 0 and ci0 + c == self.cin and ci0 % 32 == 0):
            return False
        if self.cin % 64 != 0 and c % 64 == 0:
            return True
        skip = self._skip_member(ci0)
        return skip is not None and self._defer_skip(skip, n)

    def _weight_and_input_grads(self, n, P, par, dz, part2, rows):
        e = self.eng
        cout = self.cout
        db = e.g(self.conv.name + "/bias")
        dw = e.g(self.conv.name + "/kernel")
        psum = None
        if par:
            ops.colsum(part2, rows, 4 * cout, 4, db)
            psum = torch.empty(4 * cout, device=e.device, dtype=torch.float32)
            ops.colsum(part2, rows, 4 * cout, 1, psum)
        else:
            ops.colsum(part2, rows, cout, 1, db)
        # The weight gradient is off the critical path (dz -> dgrad -> next BN backward), but
        # it stays on the compute stream: every kernel here is persistent (one workgroup per
        # CU), so a side stream only interleaves whole CUs; it measured 195.8 (one stream) vs
        # 195.6 frames/s (profiles/r03c_*) and was removed in round 6.
        targets = self._sum_targets() if self.fold_active else []
        fz = self._fused_target(n, targets)
        raw = torch.empty_like(dw) if targets else None
        if self.kind == "c3in" and self.direct:
            ops.conv_c3_wgrad(e.dt, e.x_in, n, e.h_valid, self.vout.h, self.vout.w, dz, dw)
        elif self.kind == "c3in":
            ops.conv_wgrad(e.dt, 1, ops.View(self.cols, n, self.vout.h, self.vout.w, 32, 32), dz, cout,
                           dw, dw_cols=27)
        elif self.kind == "c3":
            fold = None
            if self.fold_active:
                h, w = self.vout.h, self.vout.w
                brows = ops.border_rows(n)
                bpart = torch.empty(brows * 8 * cout, device=e.device, dtype=torch.float32)
                ops.border_sums(e.dt, dz, n, h, w, cout, bpart)
                bsum = torch.empty(8 * cout, device=e.device, dtype=torch.float32)
                ops.colsum(bpart, brows, 8 * cout, 1, bsum)
                fold = self.vin.coef() + (db, bsum)
            if self.vin.split:
                a, b = self.vin.members
                ops.conv_wgrad_cat(e.dt, a.view(n), b.view(n), dz, cout, dw, fold=fold, raw=raw)
            else:
                ops.conv_wgrad(e.dt, 9, self.vin.view(n), dz, cout, dw, fold=fold, raw=raw)
            for m, ci0 in targets:
                pm = torch.empty(L.CONSUMER_ROWS * 2 * m.c, device=e.device, dtype=torch.float32)
                ops.bn_consumer_sums(1, e.p(self.conv.name + "/kernel"), raw, cout, self.cin, ci0, m.c, db,
                                     bsum, m.producer.smean, m.producer.sinv, pm)
                m.bn_contrib.append(pm)
        else:
            fold = self.vin.coef() + (psum,) if par else None
            ops.tconv_wgrad(e.dt, self.vin.view(n), dz, cout, dw, fold=fold, raw=raw)
            for m, ci0 in targets:
                pm = torch.empty(L.CONSUMER_ROWS * 2 * m.c, device=e.device, dtype=torch.float32)
                ops.bn_consumer_sums(2, e.p(self.conv.name + "/kernel"), raw, cout, self.cin, ci0, m.c, None,
                                     psum, m.producer.smean, m.producer.sinv, pm)
                m.bn_contrib.append(pm)
        if fz is not None:
            m, ci0, frows = fz
            prod = m.producer
            coef = prod.bn_coef(n)
            whole = ci0 == 0 and m.c == self.cin
            split = self.kind == "c3" and self._split_fused(ci0, m.c, n)
            skip = self._skip_member(ci0) if split else None
            dx = None
            if not whole:
                if self.vin.ginit:
                    raise NotImplementedError(f"{self.name}: input gradient would need accumulation")
                if skip is None:
                    self.vin.ensure_grad(n, e.tdtype, e.device)
                    dx = self.vin.gview(n)
            ppar = prod.fold_active and prod.kind == "t2"
            pin = n * self.vin.h * self.vin.w
            dzp = torch.empty(pin * m.c, dtype=e.tdtype, device=e.device)
            pp = torch.empty(frows * (4 if ppar else 1) * m.c, device=e.device, dtype=torch.float32)
            if split:
                h, w = self.vout.h, self.vout.w
                if skip is not None and self._defer_skip(skip, n):
                    # the skip member's gradient is computed later, inside its producer's BN
                    # backward, together with its pool's routed gradient (_bn_backward)
                    skip.gdefer = (dz, h, w, cout, self.w_bwd)
                else:
                    if skip is not None:  # dense skip gradient: full-line traffic for the pool / BN backward
                        skip.gsep = True
                        skip.ensure_grad(n, e.tdtype, e.device)
                        dxs = skip.gview(n)
                    else:
                        dxs = ops.View(dx.buf, n, h, w, ci0, dx.ld, dx.off)
                    ops.conv3x3_dgrad(e.dt, dz, n, h, w, cout, self.w_bwd, ci0, dxs)
                wsub = self.w_bwd[ci0 * 9 * cout:]  # flipped weights [cin][3][3][cout]: rows ci0..
                ops.conv3x3_dgrad_bn(e.dt, dz, n, h, w, cout, wsub, m.c, None, 0, m.c, coef, prod.r, dzp, pp, ppar)
            elif self.kind == "c3":
                ops.conv3x3_dgrad_bn(e.dt, dz, n, self.vout.h, self.vout.w, cout, self.w_bwd, self.cin, dx, ci0,
                                     ci0 + m.c, coef, prod.r, dzp, pp, ppar)
            else:
                ops.tconv_dgrad_bn(e.dt, dz, n, self.vin.h, self.vin.w, cout, self.w_bwd, self.cin, coef, prod.r,
                                   dzp, pp)
            prod.fused = (dzp, pp, frows)
            if not whole:
                if self.vin.place:
                    self.vin.ginit = True
                else:
                    self.vin.mark_grad()
        elif self.vin.needs_grad:
            if self.vin.ginit:
                raise NotImplementedError(f"{self.name}: input gradient would need accumulation")
            self.vin.ensure_grad(n, e.tdtype, e.device)
            dx = self.vin.gview(n)
            if self.kind == "c3":
                ops.conv3x3_dgrad(e.dt, dz, n, self.vout.h, self.vout.w, cout, self.w_bwd, self.cin, dx)
            else:
                if dx.ld != dx.c or dx.off:
                    raise NotImplementedError("tconv input gradient into a concat slice")
                ops.tconv_dgrad(e.dt, dz, n, self.vin.h, self.vin.w, cout, self.w_bwd, self.cin, dx.buf)
            if self.vin.place:
                self.vin.ginit = True  # only this slice was written
            else:
                self.vin.mark_grad()
        self.r = None
        self.cols = None


class PoolStage(Stage):
    def __init__(self, layer, vin, vout):
        self.layer, self.vin, self.vout, self.name = layer, vin, vout, layer.name

    fused = False  # the producer's epilogue pools (Engine._plan_pool_fusion)

    def forward(self, n, training):
        e = self.eng
        if self.vout.place:
            raise NotImplementedError("MaxPooling2D output feeding a concatenate")
        if self.fused:
            return  # written by the producer's conv3x3_fwd_pool (pooled value + window indices)
        self.vout.ensure(n, e.tdtype, e.device)
        self.idx = torch.empty(n * self.vout.h * self.vout.w * self.vout.c, dtype=torch.uint8, device=e.device)
        aff = self.vin.coef() if training and self.vin.folded else None
        ops.maxpool_fwd(e.dt, self.vin.view(n), self.vout.buf, self.idx, aff)

    def backward(self, n):
        e = self.eng
        if not self.vin.needs_grad:
            return
        v = self.vin
        if v.sum_consumers and v.ginit:
            # this pool's share of the BN-backward sums of its input; the routing itself is
            # deferred into the producer's BN apply (cnnitmo_bn_bwd_apply_pooled)
            pp = n * (v.h // 2) * (v.w // 2)
            rows = ops.bn_bwd_rows(pp, v.c)
            pm = torch.empty(rows * 2 * v.c, device=e.device, dtype=torch.float32)
            if self.fused:  # the pooled value IS r at the window index
                ops.pool_bnsums_pooled(e.dt, self.vout.gbuf, self.vout.buf, n, v.h, v.w, v.c, v.producer.smean,
                                       v.producer.sinv, pm)
            else:
                ops.pool_bnsums(e.dt, self.vout.gbuf, self.idx, v.view(n), v.producer.smean, v.producer.sinv, pm)
            v.bn_contrib.append(pm)
            v.pool_route = (self.vout.gbuf, self.idx)
        else:
            if not v.ginit:
                if v.place:
                    raise NotImplementedError("pool gradient into an uninitialised concat slice")
                v.ensure_grad(n, e.tdtype, e.device, zero=True)
            ops.maxpool_bwd(e.dt, self.vout.gbuf, self.idx, v.gview(n))
        self.idx = None


class ConcatStage(Stage):
    def __init__(self, layer, vins, vout):
        self.layer, self.vins, self.vout, self.name = layer, vins, vout, layer.name

    def forward(self, n, training):
        self.vout.ensure(n, self.eng.tdtype, self.eng.device)

    def backward(self, n):
        pass


class HeadStage(Stage):
    def __init__(self, layer, vin):
        self.layer, self.vin, self.name = layer, vin, layer.name
        self.cin = vin.c
        self.params = [(layer.name + "/kernel", (3, 1, 1, self.cin)), (layer.name + "/bias", (3,))]

    fused = False  # computed by its producer's epilogue in predict() (Engine._plan_head_fusion)

    def infer(self, n, yhat):
        e = self.eng
        if self.fused and self.vin.producer.head_ran:
            return  # (written by the producer's cnnitmo_conv3x3_fwd_head in this forward)
        ops.head_fwd(e.dt, self.vin.view(n), e.h_valid, e.p(self.name + "/kernel"),
                     e.p(self.name + "/bias"), yhat)

    def _rank3(self):
        """The producer's BN backward can take the head's input gradient as its rank-3
        factor g3 (dy = g3 . W): a folded BN output (sums from the head's raw sums),
        no Dropout, consumed by the head alone."""
        v, e = self.vin, self.eng
        prod = v.producer
        return (e.training and v.folded and v.sum_consumers == 1 and not v.place and prod is not None
                and prod.bn is not None and prod.drop is None and prod.kind == "c3")

    def loss_and_grad(self, n, target, loss_acc, grad_numel=0.0):
        """grad_numel: the MSE gradient's normaliser (0: this batch's element count)."""
        e = self.eng
        P = n * self.vin.h * self.vin.w
        rows = ops.head_rows(P)
        part = torch.empty(rows * (5 + 3 * self.cin), device=e.device, dtype=torch.float32)
        aff = self.vin.coef() if e.training and self.vin.folded else None
        wt = e.p(self.name + "/kernel")
        if self._rank3():
            g3 = torch.empty(P * 3, device=e.device, dtype=torch.float32)
            ops.head_fwd_bwd_g3(e.dt, self.vin.view(n), e.h_valid, wt, e.p(self.name + "/bias"), target, g3,
                                part, aff, grad_numel)
            self.vin.grad_g3 = (g3, wt)
        else:
            self.vin.ensure_grad(n, e.tdtype, e.device)
            dx = self.vin.gview(n)
            ops.head_fwd_bwd(e.dt, self.vin.view(n), e.h_valid, wt, e.p(self.name + "/bias"), target, dx.buf,
                             part, aff, grad_numel)
        v = self.vin
        raw = torch.empty(3 * self.cin, device=e.device, dtype=torch.float32) \
            if e.training and v.sum_consumers and v.folded else None
        ops.head_finalize(part, rows, self.cin, n * e.h_valid * self.vin.w * 3, loss_acc,
                          e.g(self.name + "/kernel"), e.g(self.name + "/bias"), aff, raw=raw)
        if raw is not None:
            pm = torch.empty(L.CONSUMER_ROWS * 2 * v.c, device=e.device, dtype=torch.float32)
            ops.bn_consumer_sums(3, e.p(self.name + "/kernel"), raw, 3, self.cin, 0, v.c, e.g(self.name + "/bias"),
                                 None, v.producer.smean, v.producer.sinv, pm)
            v.bn_contrib.append(pm)
        self.vin.mark_grad()


# ---------------------------------------------------------------------------
def compile_graph(model, fold=True):
    """Turn the Keras layer graph into an ordered list of stages.  fold: keep BN
    outputs (without Dropout) unmaterialised in training (see module doc)."""
    layers = model.layers
    cons = {}
    for l in layers:
        for t in l.inbound:
            cons.setdefault(id(t), []).append(l)

    def only_consumer(t):
        c = cons.get(id(t), [])
        return c[0] if len(c) == 1 else None

    values = {}
    stages = []
    consumed = set()
    inp = model.inputs[0]
    vin = Value(inp.layer.name, inp.shape)
    vin.needs_grad = False
    values[id(inp)] = vin
    drop_count = 0
    out_t = model.outputs[0]
    for l in layers:
        if id(l) in consumed or isinstance(l, InputLayer):
            continue
        if isinstance(l, (Conv2D, Conv2DTranspose)):
            x = l.inbound[0]
            if isinstance(l, Conv2D) and l.kernel_size == (1, 1) and l.activation == "sigmoid":
                if l.output is not out_t:
                    raise NotImplementedError("a 1x1 sigmoid conv is supported only as the model head")
                stages.append(HeadStage(l, values[id(x)]))
                continue
            if isinstance(l, Conv2D) and not (l.kernel_size == (3, 3) and l.padding == "same"):
                raise NotImplementedError(f"{l.name}: only 3x3 'same' convs (and the 1x1 sigmoid head)")
            t = l.output
            relu = l.activation == "relu"
            if l.activation not in (None, "relu"):
                raise NotImplementedError(f"{l.name}: activation {l.activation}")
            nxt = only_consumer(t)
            if not relu and isinstance(nxt, Activation) and nxt.activation == "relu":
                consumed.add(id(nxt))
                relu = True
                t = nxt.output
                nxt = only_consumer(t)
            if not relu:
                raise NotImplementedError(f"{l.name}: conv without ReLU is not on the path")
            bn = None
            if isinstance(nxt, BatchNormalization):
                bn = nxt
                consumed.add(id(bn))
                t = bn.output
                nxt = only_consumer(t)
            drop = None
            drop_id = 0
            if isinstance(nxt, Dropout):
                if bn is None:
                    raise NotImplementedError("Dropout without a preceding BatchNormalization")
                drop = nxt
                consumed.add(id(drop))
                drop_count += 1
                drop_id = drop_count  # ordinal of the Dropout in the model (1, 2): hash layer id
                t = drop.output
            if isinstance(l, Conv2DTranspose):
                if bn is None:
                    raise NotImplementedError("Conv2DTranspose without BN is not on the path")
                kind = "t2"
            elif x is inp and inp.shape[-1] == 3:
                kind = "c3in"
            else:
                kind = "c3"
            vout = Value(t.layer.name, t.shape)
            vout.folded = fold and bn is not None and drop is None
            values[id(t)] = vout
            st = BlockStage(kind, l, relu, bn, drop, drop_id, values[id(x)], vout)
            vout.producer = st
            stages.append(st)
        elif isinstance(l, MaxPooling2D):
            vout = Value(l.name, l.output.shape)
            values[id(l.output)] = vout
            stages.append(PoolStage(l, values[id(l.inbound[0])], vout))
        elif isinstance(l, Concatenate):
            vout = Value(l.name, l.output.shape)
            values[id(l.output)] = vout
            off = 0
            vins = []
            for t in l.inbound:
                v = values[id(t)]
                if v.place is not None or v is vin or v.members:
                    raise NotImplementedError(f"{l.name}: input {v.name} cannot be placed zero-copy")
                v.place = (vout, off)
                vout.members.append(v)
                off += v.c
                vins.append(v)
            vout.folded = any(v.folded for v in vins)
            stages.append(ConcatStage(l, vins, vout))
        else:
            raise NotImplementedError(f"{l.name} ({type(l).__name__}) outside a fusable pattern")
    if not stages or not isinstance(stages[-1], HeadStage):
        raise NotImplementedError("the model must end in Conv2D(3, 1, activation='sigmoid')")
    _plan_bn_sums(stages)
    return stages


def _plan_bn_sums(stages):
    """Mark the folded BN outputs whose backward sums (sum dy, sum dy*rhat) can be
    assembled from their consumers instead of a pass over dy: every consumer must be a
    conv3x3 / tconv / head (cnnitmo_bn_consumer_sums) or a MaxPooling2D
    (cnnitmo_maxpool2x2_bwd_bnsums).  Dropout outputs are materialised, hence never folded."""
    readers = {}
    for st in stages:
        srcs = []
        if isinstance(st, (BlockStage, PoolStage, HeadStage)):
            srcs = [st.vin]
        for v in srcs:
            for m in (v.members if v.members else [v]):
                readers.setdefault(id(m), []).append(st)
    for st in stages:
        if not isinstance(st, BlockStage) or st.bn is None or st.drop is not None:
            continue
        v = st.vout
        if not v.folded:
            continue
        rs = readers.get(id(v), [])
        ok = bool(rs) and all(
            (isinstance(r, BlockStage) and r.kind in ("c3", "t2")) or isinstance(r, (PoolStage, HeadStage))
            for r in rs)
        v.sum_consumers = len(rs) if ok else 0
        v.fuse_into = rs[0] if (ok and len(rs) == 1 and isinstance(rs[0], BlockStage) and
                                rs[0].kind in ("c3", "t2")) else None


def layout_params(stages):
    """Flat fp32 layout of every trainable tensor in REVERSE stage order (backward
    writes gradients front to back).  Returns (pslices, bslices, stage_goff,
    nparams, nbuffers); stage_goff[i] = [lo, hi) gradient range of stages[i]."""
    pslices, bslices, ranges = {}, {}, {}
    off = boff = 0
    for st in reversed(stages):
        lo = off
        for k, shp in st.params:
            n = int(np.prod(shp))
            pslices[k] = (off, shp)
            off += -(-n // ALIGN) * ALIGN
        ranges[id(st)] = (lo, off)
        for k, shp in st.buffers:
            n = int(np.prod(shp))
            bslices[k] = (boff, shp)
            boff += n
    return pslices, bslices, [ranges[id(s)] for s in stages], off, boff


class Engine:
    """Runtime for one compiled model on one GPU (one process per GPU)."""

    def __init__(self, model, dtype="float32", device="cuda"):
        if not torch.cuda.is_available():
            raise L.CnnItmoError("the CNN-ITMO engine needs a ROCm GPU (no CPU fallback)")
        L.load()
        self.model = model
        self.dtype_name = dtype
        self.dt, self.tdtype = ops.DTYPES[dtype]
        self.device = torch.device(device)
        self.stages = compile_graph(model)
        self._plan_split_concats()
        self._plan_pool_fusion()
        self._plan_head_fusion()
        self._yhat = None
        self.training = False
        self.h_valid = None
        self.update_moving = True
        self.drop_seed = 0
        self.pslices, self.bslices, self.stage_goff, off, boff = layout_params(self.stages)
        self.nparams = off
        self.params = torch.zeros(off, device=self.device, dtype=torch.float32)
        self.grads = torch.zeros(off, device=self.device, dtype=torch.float32)
        self.accum = torch.zeros(off, device=self.device, dtype=torch.float32)
        self.bufs = torch.zeros(max(boff, 1), device=self.device, dtype=torch.float32)
        for st in self.stages:
            st.bind(self)
        self.weights_dirty = True
        self.step = 0
        self.grad_hook = None  # callable(lo, hi) after each stage's gradients are written
        self.fwd_hook = None  # callable() after the training forward (moving stats final)

    def _plan_split_concats(self):
        """Keep the members of a concatenate in dense buffers of their own when their
        slices of a concat row would cover partial 128-B lines: the level-0 concat
        [conv1 32 | up9 64] (model.py:261) puts 64 + 128 B of each 192-B row in lines
        shared with the neighbouring pixels, so the pool, its BN-sum pass and enc1b's
        BN-backward apply read conv1 in half lines and up9 writes them.  Its consumer
        (conv9, a 3x3 conv, model.py:262) then reads both members directly: cnnitmo_conv3x3_fwd_cat /
        cnnitmo_conv_wgrad_cat (bf16 halo kernels; its input gradient is already split
        per member).  Sizes either entry point rejects: one concat buffer."""
        if self.dt != L.BF16:
            return
        readers = {}
        for st in self.stages:
            for v in [getattr(st, "vin", None)]:
                if v is not None:
                    readers.setdefault(id(v), []).append(st)
        for st in self.stages:
            if not isinstance(st, ConcatStage):
                continue
            v = st.vout
            rs = readers.get(id(v), [])
            if len(v.members) != 2 or len(rs) != 1 or not isinstance(rs[0], BlockStage) or rs[0].kind != "c3":
                continue
            c1, c = v.members[0].c, v.c
            esz = 2  # bf16
            if (c1 * esz) % 128 == 0 and (c * esz) % 128 == 0:
                continue  # member slices already cover whole lines
            # both halves must run on the split members: the forward (bf16 halo kernel,
            # which CNNITMO_HALO=0 or a small device rules out) and the weight gradient
            if not (ops.fwd_cat_supported(self.dt, 1, v.h, v.w, c1, c, rs[0].cout)
                    and ops.wgrad_cat_supported(1, v.h, v.w, c1, c, rs[0].cout)):
                continue
            v.split = True

    def _plan_pool_fusion(self):
        """MaxPooling2D into its producer's epilogue (model.py:209-220: ConvBN -> pool at
        levels 0-2): the conv3x3 whose BN output the pool reads writes the pooled value and
        window indices itself (cnnitmo_conv3x3_fwd_pool), which removes the pool's re-read of
        the full-resolution output.  In training the producer stores r (BN folded into its
        consumers) and pools r by sign(gamma); the pooled value is then a folded value too,
        with the producer's BN coefficients (Value.coef_src), and its consumer conv folds them
        like any other.  Needs: a 'c3' producer with BN and no Dropout (Dropout outputs are
        materialised by bn_apply), BN folding on, the halo kernel for the producer's sizes
        (otherwise the stand-alone pool kernel)."""
        for st in self.stages:
            if not isinstance(st, PoolStage):
                continue
            v = st.vin
            prod = v.producer
            if (prod is None or prod.kind != "c3" or prod.bn is None or prod.drop is not None or not v.folded
                    or v.split or prod.vin.split or st.vout.place):
                continue
            if not ops.pool_supported(self.dt, 1, v.h, v.w, prod.vin.c if prod.kind == "c3" else 3, prod.cout):
                continue
            st.fused = True
            prod.pool = st
            st.vout.folded = True
            st.vout.coef_src = v

    def _plan_head_fusion(self):
        """The sigmoid head (model.py:276) into the inference epilogue of the 3x3 ConvBN that
        feeds it (conv9, model.py:262): predict() then never stores that conv's 64-channel
        output (fp32 b8 at 1080p: 4.3 GB written and read back).  Needs: a 'c3' producer with
        BN and no Dropout / pooling / concat, consumed by the head alone, 64 channels, the halo
        kernel for its sizes (otherwise the stand-alone head kernel)."""
        head = self.stages[-1]
        if not isinstance(head, HeadStage):
            return
        v = head.vin
        prod = v.producer
        readers = sum(1 for st in self.stages if getattr(st, "vin", None) is v or v in getattr(st, "vins", []))
        if (prod is None or not isinstance(prod, BlockStage) or prod.kind != "c3" or prod.bn is None
                or prod.drop is not None or prod.pool is not None or v.place or v.split or prod.vin.split
                or readers != 1 or prod.cout != 64 or head.cin != 64):
            return
        if not ops.head_supported(self.dt, 1, v.h, v.w, prod.cin, prod.cout):
            return
        prod.head = head
        head.fused = True

    # ---- parameter access ---------------------------------------------------
    def _slice(self, flat, table, key):
        off, shp = table[key]
        return flat[off:off + int(np.prod(shp))]

    def p(self, key):
        return self._slice(self.params, self.pslices, key)

    def g(self, key):
        return self._slice(self.grads, self.pslices, key)

    def b(self, key):
        return self._slice(self.bufs, self.bslices, key)

    def set_weights(self, named):
        for k, v in named.items():
            t = torch.as_tensor(np.ascontiguousarray(v, dtype=np.float32).reshape(-1))
            if k in self.pslices:
                self.p(k).copy_(t)
            elif k in self.bslices:
                self.b(k).copy_(t)
            else:
                raise KeyError(k)
        self.weights_dirty = True

    def get_weights(self):
        out = {}
        for k, (_, shp) in self.pslices.items():
            out[k] = self.p(k).cpu().numpy().reshape(shp).copy()
        for k, (_, shp) in self.bslices.items():
            out[k] = self.b(k).cpu().numpy().reshape(shp).copy()
        return out

    def get_grads(self):
        return {k: self.g(k).cpu().numpy().reshape(shp).copy() for k, (_, shp) in self.pslices.items()}

    def prepare_weights(self):
        if self.weights_dirty:
            for st in self.stages:
                if isinstance(st, BlockStage):
                    st.prep()
            self.weights_dirty = False

    # ---- execution ----------------------------------------------------------
    def _input(self, x):
        """x: [n, h_valid, w, 3] fp32 device tensor; pads H to the model's height."""
        n, hv, w, c = x.shape
        vin = self.stages[0].vin if isinstance(self.stages[0], BlockStage) else None
        H, W, C = self.model.inputs[0].shape
        if c != 3 or w != W or hv > H or H - hv >= 16:
            raise ValueError(f"input of shape {tuple(x.shape)} does not fit model input (None, {H}, {W}, {C})")
        self.x_in = x.contiguous().float()
        self.h_valid = hv
        return n

    def _release(self):
        seen = set()
        for st in self.stages:
            for v in [getattr(st, "vout", None), getattr(st, "vin", None)] + list(getattr(st, "vins", [])):
                if v is not None and id(v) not in seen:
                    seen.add(id(v))
                    v.release()

    def forward(self, x, training=False):
        n = self._input(x)
        self.prepare_weights()
        self.training = training
        for st in self.stages[:-1]:
            st.forward(n, training)
        return n

    def predict(self, x):
        # [n, h_valid, w, 3]: x's valid rows (forward's _input)
        yhat = torch.empty(x.shape[0], x.shape[1], self.model.inputs[0].shape[1], 3, device=self.device,
                           dtype=torch.float32)
        return self.predict_into(x, yhat)

    def predict_into(self, x, yhat):
        """predict() into a caller's fp32 [n, h_valid, w, 3] buffer (bench.py's inference legs
        reuse one).  A fused head writes it from its producer's epilogue during the forward."""
        if tuple(yhat.shape) != (x.shape[0], x.shape[1], self.model.inputs[0].shape[1], 3) or \
                yhat.dtype != torch.float32 or not yhat.is_contiguous():
            raise ValueError(f"predict_into: yhat must be contiguous fp32 {(x.shape[0], x.shape[1])} x W x 3, "
                             f"got {tuple(yhat.shape)} {yhat.dtype}")
        self._yhat = yhat
        try:
            n = self.forward(x, training=False)
        finally:
            self._yhat = None
        self.stages[-1].infer(n, yhat)
        self._release()
        return yhat

    def train_step(self, x, target, seed=None, lr=1e-3, rho=0.9, eps=1e-7, grad_scale=1.0,
                   sync=None, apply=True, grad_frames=None):
        """One fwd+bwd+RMSprop step.  Returns a device tensor [loss, acc] (this batch's means).
        grad_frames: the frame count the loss gradient is normalised by (default: this
        batch's).  Data parallel with unequal shares, global_frames / world makes the
        averaged gradient that of the global batch mean (Model.train_on_batch)."""
        if x.shape[0] == 0:
            raise ValueError("train_step: empty batch (BatchNormalization statistics of zero frames)")
        self.drop_seed = self.step if seed is None else int(seed)
        n = self.forward(x, training=True)
        if self.fwd_hook:
            self.fwd_hook()
        loss_acc = torch.empty(2, device=self.device, dtype=torch.float32)
        head = self.stages[-1]
        gn = 0.0 if grad_frames is None else float(grad_frames) * self.h_valid * self.model.inputs[0].shape[1] * 3
        head.loss_and_grad(n, target.contiguous().float(), loss_acc, gn)
        if self.grad_hook:  # (DP all-reduce launches behind the stage's gradient writes)
            self.grad_hook(*self.stage_goff[-1])
        for i in range(len(self.stages) - 2, -1, -1):
            st = self.stages[i]
            st.backward(n)
            if self.grad_hook and st.params:
                self.grad_hook(*self.stage_goff[i])
        self._release()
        if sync is not None:
            sync()
        if apply:
            ops.rmsprop(self.params, self.grads, self.accum, lr, rho, eps, grad_scale)
            self.weights_dirty = True
        self.step += 1
        return loss_acc

    def evaluate_batch(self, x, target):
        n = self.forward(x, training=False)
        loss_acc = torch.empty(2, device=self.device, dtype=torch.float32)
        saved = self.grads.clone()
        self.stages[-1].loss_and_grad(n, target.contiguous().float(), loss_acc)
        self.grads.copy_(saved)
        self._release()
        return loss_acc
