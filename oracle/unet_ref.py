"""CPU oracle for the CNN-ITMO hot path -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``cnn_itmo_amd``) never imports anything from ``oracle/``.

It restates, in numpy (fp64 reference mode or fp32 timing mode), the arithmetic
that the reference delegates to Keras 2.2.x / TensorFlow 1.x:

* ``ConvBN``        -- /root/reference/model.py:195-196
                       Conv2D(f, 3, padding='same', he_normal) -> ReLU -> BatchNormalization
* ``ConvBNTranspose`` -- /root/reference/model.py:199-200
                       Conv2DTranspose(f, 2, strides=2, 'valid') -> ReLU -> BatchNormalization
* ``U_net`` graph   -- /root/reference/model.py:204-278  (pools :210,215,220,227;
                       dropouts :226,239; concats [skip, up] :246,251,256,261; head :276)
* compile           -- /root/reference/model.py:281  (rmsprop, mse, 'accuracy')
* predict I/O       -- /root/reference/predict.py:59-64 (x/255 in, (pred*255).astype(uint8) out)

Parity status: **parity unpinned** against the reference itself.  Keras/TF are
not vendored under /root/reference and cannot be imported here
(``ModuleNotFoundError: keras`` at model.py:14), the trained weights are missing
(/root/reference/.MISSING_LARGE_BLOBS:1) and the reference has no tests or golden
vectors.  What pins this restatement instead: the reference's own ``layers.txt``
(shapes + the 11,166,819 / 7,808 parameter counts, checked in tests), and an
independent cross-check of every op against torch-CPU autograd
(``tests/test_oracle.py``).  Keras-2.2 semantics restated here are marked
[Keras-2.2] and follow SURVEY.md section 8a.

Layouts (shared with the HIP path):
  activations NHWC; Conv2D kernel OHWI ``[Cout, kh, kw, Cin]``;
  Conv2DTranspose kernel ``[2, 2, Cout, Cin]`` (Keras' own layout, layers.txt:78);
  head kernel ``[3, 1, 1, 64]``.
"""
from __future__ import annotations

import numpy as np

BN_EPS = 1e-3          # Keras BatchNormalization default epsilon [Keras-2.2]
BN_MOMENTUM = 0.99     # Keras BatchNormalization default momentum [Keras-2.2]
RMS_LR = 1e-3          # keras.optimizers.RMSprop defaults [Keras-2.2]
RMS_RHO = 0.9
RMS_EPS = 1e-7         # K.epsilon(), added OUTSIDE the sqrt [Keras-2.2]
DROP_RATE = 0.5        # model.py:226,239

_M64 = (1 << 64) - 1


# --------------------------------------------------------------------------
# Dropout mask: counter-based hash shared bit-exactly with the HIP kernels
# (csrc/common.h: dropout_keep).  Keras draws from TF's RNG, which is not
# reproducible across frameworks; the keep-probability 0.5 and the x2 scale
# (inverted dropout, model.py:226,239) are what is reproduced.
# --------------------------------------------------------------------------
def dropout_keep(seed: int, layer: int, count: int, start: int = 0) -> np.ndarray:
    """Boolean keep-mask for flat element indices [start, start+count)."""
    with np.errstate(over="ignore"):
        idx = np.arange(start, start + count, dtype=np.uint64)
        base = np.uint64((seed * 0x9E3779B97F4A7C15 + layer * 0xD1B54A32D192ED03) & _M64)
        x = idx + base
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return (x >> np.uint64(63)) == 0


def dropout_fwd(y, seed, layer):
    keep = dropout_keep(seed, layer, y.size).reshape(y.shape)
    return np.where(keep, y * 2.0, 0.0).astype(y.dtype), keep


# --------------------------------------------------------------------------
# Convolutions (TF cross-correlation, no flip).  model.py:196 / :276
# --------------------------------------------------------------------------
def _im2col(xp, kh, kw, H, W, h0, h1):
    """xp: zero-padded NHWC; returns [N, h1-h0, W, kh*kw*C] for output rows h0:h1."""
    N, _, _, C = xp.shape
    cols = np.empty((N, h1 - h0, W, kh, kw, C), dtype=xp.dtype)
    for r in range(kh):
        for s in range(kw):
            cols[:, :, :, r, s, :] = xp[:, h0 + r:h1 + r, s:s + W, :]
    return cols.reshape(N, h1 - h0, W, kh * kw * C)


def _bands(H, band, fn):
    """fn(h0, h1) over the row bands [h0, h1) of H, results in band order.  Large frames run
    the bands on a thread pool (numpy releases the GIL in the im2col copies and in BLAS);
    every band's arithmetic is the same as in a sequential loop."""
    spans = [(h0, min(H, h0 + band)) for h0 in range(0, H, band)]
    if len(spans) < 4:
        return [fn(a, b) for a, b in spans]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=_POOL) as ex:
        return list(ex.map(lambda s: fn(*s), spans))


_POOL = max(1, min(8, int(__import__("os").environ.get("OMP_NUM_THREADS", "8") or 8)))


def conv2d_same(x, w, b=None, band=64):
    """Conv2D 'same', stride 1.  x [N,H,W,Ci], w OHWI [Co,kh,kw,Ci], b [Co]."""
    N, H, W, Ci = x.shape
    Co, kh, kw, _ = w.shape
    ph, pw = kh // 2, kw // 2
    xp = np.pad(x, ((0, 0), (ph, ph), (pw, pw), (0, 0)))
    wm = w.reshape(Co, -1).T  # [kh*kw*Ci, Co]
    out = np.empty((N, H, W, Co), dtype=x.dtype)

    def one(h0, h1):
        out[:, h0:h1] = _im2col(xp, kh, kw, H, W, h0, h1) @ wm
    _bands(H, band, one)
    if b is not None:
        out += b
    return out


def conv2d_same_bwd(x, w, dz, need_dx=True, band=64):
    """Gradients of conv2d_same.  Returns (dx, dw, db)."""
    N, H, W, Ci = x.shape
    Co, kh, kw, _ = w.shape
    ph, pw = kh // 2, kw // 2
    db = dz.reshape(-1, Co).sum(0)
    xp = np.pad(x, ((0, 0), (ph, ph), (pw, pw), (0, 0)))
    dw = np.zeros((kh * kw * Ci, Co), dtype=x.dtype)
    parts = _bands(H, band, lambda h0, h1: _im2col(xp, kh, kw, H, W, h0, h1).reshape(-1, kh * kw * Ci).T
                   @ dz[:, h0:h1].reshape(-1, Co))
    for pt in parts:  # summed in band order, as a sequential loop would
        dw += pt
    dw = dw.T.reshape(Co, kh, kw, Ci)
    dx = None
    if need_dx:
        # dx = conv_same(dz, W') with W'[ci, r', s', co] = W[co, kh-1-r', kw-1-s', ci]
        wf = np.ascontiguousarray(w[:, ::-1, ::-1, :].transpose(3, 1, 2, 0))
        dx = conv2d_same(dz, wf, None, band)
    return dx, dw, db


def tconv2x2s2(x, k, b=None):
    """Conv2DTranspose(f, 2, strides=2, 'valid') -- model.py:200.

    out[n, 2i+a, 2j+c, co] = sum_ci x[n,i,j,ci] * k[a,c,co,ci] + b[co]
    """
    N, H, W, Ci = x.shape
    Co = k.shape[2]
    t = np.einsum("nhwi,abOi->nhawbO", x, k, optimize=True)  # [N,H,2,W,2,Co]
    out = t.reshape(N, 2 * H, 2 * W, Co)
    if b is not None:
        out = out + b
    return out


def tconv2x2s2_bwd(x, k, dout):
    """dx[n,h,w,i] = sum_{a,b,O} dout[n,2h+a,2w+b,O] k[a,b,O,i];  dk[a,b,O,i] = sum_{n,h,w}
    dout[n,2h+a,2w+b,O] x[n,h,w,i] -- one GEMM per tap (a, b)."""
    N, H, W, Ci = x.shape
    Co = k.shape[2]
    d = dout.reshape(N, H, 2, W, 2, Co)
    x2 = x.reshape(-1, Ci)
    dx = np.zeros((N * H * W, Ci), dtype=np.result_type(dout, k))
    dk = np.empty((2, 2, Co, Ci), dtype=np.result_type(dout, x))
    for a in range(2):
        for b in range(2):
            dt = np.ascontiguousarray(d[:, :, a, :, b, :]).reshape(-1, Co)
            dx += dt @ k[a, b]
            dk[a, b] = dt.T @ x2
    db = dout.reshape(-1, Co).sum(0)
    return dx.reshape(N, H, W, Ci), dk, db


# --------------------------------------------------------------------------
# MaxPooling2D(2, strides=2) 'valid' -- model.py:210,215,220,227.
# Tie rule (unpinned upstream; fixed here and in the HIP kernel): gradient goes
# to the FIRST maximum in row-major window order (0,0),(0,1),(1,0),(1,1).
# --------------------------------------------------------------------------
def maxpool2x2(x):
    N, H, W, C = x.shape
    Ho, Wo = H // 2, W // 2
    v = x[:, :2 * Ho, :2 * Wo].reshape(N, Ho, 2, Wo, 2, C).transpose(0, 1, 3, 2, 4, 5)
    v = v.reshape(N, Ho, Wo, 4, C)
    idx = np.argmax(v, axis=3)  # numpy argmax returns first max
    y = np.take_along_axis(v, idx[:, :, :, None, :], axis=3)[:, :, :, 0, :]
    return y, idx.astype(np.uint8)


def maxpool2x2_bwd(dy, idx, in_shape):
    N, H, W, C = in_shape
    Ho, Wo = H // 2, W // 2
    d = np.zeros((N, Ho, Wo, 4, C), dtype=dy.dtype)
    np.put_along_axis(d, idx[:, :, :, None, :].astype(np.int64), dy[:, :, :, None, :], axis=3)
    d = d.reshape(N, Ho, Wo, 2, 2, C).transpose(0, 1, 3, 2, 4, 5).reshape(N, 2 * Ho, 2 * Wo, C)
    out = np.zeros(in_shape, dtype=dy.dtype)
    out[:, :2 * Ho, :2 * Wo] = d
    return out


# --------------------------------------------------------------------------
# BatchNormalization (axis=-1) -- model.py:196,200 [Keras-2.2]
# --------------------------------------------------------------------------
def bn_train_fwd(r, gamma, beta, eps=BN_EPS):
    C = r.shape[-1]
    rf = r.reshape(-1, C)
    mean = rf.mean(0)
    var = rf.var(0)  # biased (tf.nn.moments)
    invstd = 1.0 / np.sqrt(var + eps)
    y = (r - mean) * (gamma * invstd) + beta
    return y, mean, var


def bn_infer(r, gamma, beta, mmean, mvar, eps=BN_EPS):
    return (r - mmean) * (gamma / np.sqrt(mvar + eps)) + beta


def bn_moving_update(mmean, mvar, mean, var, count, momentum=BN_MOMENTUM, eps=BN_EPS):
    """Moving-statistics update of keras BatchNormalization.call in training
    [Keras-2.2 + TF-1.x semantics, model.py:196,200]:
    * K.normalize_batch_in_training takes ``_fused_normalize_batch_in_training``
      (tf.nn.fused_batch_norm) for 4-D NHWC input; the fused op normalises with the
      biased variance but RETURNS the Bessel-corrected batch variance n/(n-1)*var;
    * Keras then applies ``variance *= n / (n - (1 + eps))`` on top;
    * K.moving_average_update: x <- x*momentum + v*(1-momentum)."""
    var_u = var * (count / (count - 1.0)) * (count / (count - (1.0 + eps)))
    return mmean * momentum + mean * (1 - momentum), mvar * momentum + var_u * (1 - momentum)


def bn_train_bwd(dy, r, gamma, mean, var, eps=BN_EPS):
    C = r.shape[-1]
    M = r.size // C
    invstd = 1.0 / np.sqrt(var + eps)
    rhat = (r - mean) * invstd
    dyf = dy.reshape(-1, C)
    sdy = dyf.sum(0)
    sdyr = (dyf * rhat.reshape(-1, C)).sum(0)
    dr = (gamma * invstd / M) * (M * dy - sdy - rhat * sdyr)
    return dr, sdyr, sdy  # dr, dgamma, dbeta


# --------------------------------------------------------------------------
# Head / loss / metric / optimizer -- model.py:276,281
# --------------------------------------------------------------------------
def sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def mse(yhat, t):
    return float(np.mean((yhat - t) ** 2))


def mse_grad_z(yhat, t):
    """d(mean((sigmoid(z)-t)^2))/dz."""
    return 2.0 * (yhat - t) * yhat * (1.0 - yhat) / yhat.size


def categorical_accuracy(t, yhat):
    """Keras 'accuracy' with a 3-channel output -> categorical_accuracy [Keras-2.2]."""
    return float(np.mean(np.argmax(t, -1) == np.argmax(yhat, -1)))


def rmsprop(p, g, a, lr=RMS_LR, rho=RMS_RHO, eps=RMS_EPS):
    a_new = rho * a + (1.0 - rho) * g * g
    p_new = p - lr * g / (np.sqrt(a_new) + eps)
    return p_new, a_new


# --------------------------------------------------------------------------
# The U-Net (model.py:204-278) and the config-1 3-conv net
# --------------------------------------------------------------------------
ENC = [32, 64, 128, 256]
CROSS = 512
DEC = [512, 256, 128, 64]

# Conv layer table in Keras creation order (layers.txt): name, kind, cin, cout
UNET_LAYERS = [
    ("conv2d_1", "c3", 3, 32), ("conv2d_2", "c3", 32, 32),
    ("conv2d_3", "c3", 32, 64), ("conv2d_4", "c3", 64, 64),
    ("conv2d_5", "c3", 64, 128), ("conv2d_6", "c3", 128, 128),
    ("conv2d_7", "c3", 128, 256), ("conv2d_8", "c3", 256, 256),
    ("conv2d_9", "c3", 256, 512), ("conv2d_10", "c3", 512, 512),
    ("conv2d_transpose_1", "t2", 512, 512), ("conv2d_11", "c3", 768, 512),
    ("conv2d_transpose_2", "t2", 512, 256), ("conv2d_12", "c3", 384, 256),
    ("conv2d_transpose_3", "t2", 256, 128), ("conv2d_13", "c3", 192, 128),
    ("conv2d_transpose_4", "t2", 128, 64), ("conv2d_14", "c3", 96, 64),
    ("conv2d_15", "c1", 64, 3),
]


def truncated_normal(rng, shape):
    """tf.truncated_normal(mean 0, stddev 1): standard normal values, every value
    outside [-2, 2] re-drawn until it falls inside (Keras 2.2 he_normal ->
    VarianceScaling(distribution='normal') -> K.truncated_normal)."""
    z = rng.standard_normal(shape)
    bad = np.abs(z) > 2.0
    while bad.any():
        z[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(z) > 2.0
    return z


def init_unet_params(seed=0, dtype=np.float64):
    """Seeded init with Keras' *distributions* (he_normal truncated, glorot_uniform
    for the head, zero biases, BN gamma=1 beta=0, moving 0/1).  Keras' exact RNG
    stream is not reproducible outside TF, so init is statistically pinned only."""
    rng = np.random.default_rng(seed)
    P = {}
    bn_i = 1
    for name, kind, ci, co in UNET_LAYERS:
        if kind == "c3":
            fan_in = 9 * ci
            std = np.sqrt(2.0 / fan_in) / 0.87962566103423978
            w = truncated_normal(rng, (co, 3, 3, ci)) * std
        elif kind == "t2":
            fan_in = 4 * co  # Keras _compute_fans on (2,2,Cout,Cin): fan_in = Cout*4
            std = np.sqrt(2.0 / fan_in) / 0.87962566103423978
            w = truncated_normal(rng, (2, 2, co, ci)) * std
        else:
            lim = np.sqrt(6.0 / (ci + co))
            w = rng.uniform(-lim, lim, (co, 1, 1, ci))
        P[name + "/kernel"] = w.astype(dtype)
        P[name + "/bias"] = np.zeros(co, dtype)
        if kind != "c1":
            bn = f"batch_normalization_{bn_i}"
            bn_i += 1
            P[bn + "/gamma"] = np.ones(co, dtype)
            P[bn + "/beta"] = np.zeros(co, dtype)
            P[bn + "/moving_mean"] = np.zeros(co, dtype)
            P[bn + "/moving_variance"] = np.ones(co, dtype)
    return P


def bn_name_for(conv_name):
    order = [n for n, k, _, _ in UNET_LAYERS if k != "c1"]
    return f"batch_normalization_{order.index(conv_name) + 1}"


def round_bf16(a):
    """Round to the nearest bfloat16 (ties to even), returned as float64."""
    u = np.asarray(a, np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


class UNetRef:
    """Forward/backward of the U-Net exactly as model.py:204-278 wires it.

    ``bn_groups``: the batch is split into that many equal groups with
    independent BN batch statistics -- the per-replica BN of data parallelism
    (SURVEY.md 8e).

    ``store``: optional rounding applied wherever a tensor is STORED in a
    reduced-precision pipeline (e.g. ``round_bf16``): the network input, the
    conv / transposed-conv weights, every post-ReLU activation and BN output,
    and every input-gradient / pre-activation gradient in the backward.  The
    arithmetic itself stays in ``dtype``.  It emulates bf16 storage with fp32
    accumulation, giving the noise floor a bf16 implementation is held to."""

    def __init__(self, params, dtype=np.float64, store=None):
        self.P = {k: np.asarray(v, dtype) for k, v in params.items()}
        self.dtype = dtype
        self.q = store if store is not None else (lambda a: a)

    # ----- building blocks -------------------------------------------------
    def _convbn(self, name, x, training, kind, groups, cache):
        P = self.P
        bn = bn_name_for(name)
        w, b = self.q(P[name + "/kernel"]), P[name + "/bias"]
        z = conv2d_same(x, w, b) if kind == "c3" else tconv2x2s2(x, w, b)
        r = self.q(np.maximum(z, 0))
        g, be = P[bn + "/gamma"], P[bn + "/beta"]
        if training:
            ys, stats = [], []
            for rr in np.split(r, groups, axis=0):
                y, m, v = bn_train_fwd(rr, g, be)
                ys.append(y)
                stats.append((m, v, rr.size // rr.shape[-1]))
            y = np.concatenate(ys, 0)
        else:
            y = bn_infer(r, g, be, P[bn + "/moving_mean"], P[bn + "/moving_variance"])
            stats = None
        cache[name] = dict(x=x, r=r, stats=stats, kind=kind, bn=bn)
        return self.q(y)

    def forward(self, x, training=False, seed=0, groups=1, drop_seeds=None):
        """x: [N,H,W,3] in [0,1].  Returns sigmoid output.  ``drop_seeds`` gives
        per-group dropout seeds (default: seed for all groups)."""
        x = self.q(np.asarray(x, self.dtype))
        c = {}
        self.cache = c
        self.training = training
        self.groups = groups
        if drop_seeds is None:
            drop_seeds = [seed] * groups
        self.drop_seeds = drop_seeds

        def drop(y, layer):
            if not training:
                return y, None
            parts, keeps = [], []
            for gi, yy in enumerate(np.split(y, groups, axis=0)):
                o, k = dropout_fwd(yy, drop_seeds[gi], layer)
                parts.append(o)
                keeps.append(k)
            return np.concatenate(parts, 0), np.concatenate(keeps, 0)

        cb = lambda n, t: self._convbn(n, t, training, "c3", groups, c)
        tb = lambda n, t: self._convbn(n, t, training, "t2", groups, c)
        conv1 = cb("conv2d_2", cb("conv2d_1", x))
        pool1, c["pool1"] = maxpool2x2(conv1)
        conv2 = cb("conv2d_4", cb("conv2d_3", pool1))
        pool2, c["pool2"] = maxpool2x2(conv2)
        conv3 = cb("conv2d_6", cb("conv2d_5", pool2))
        pool3, c["pool3"] = maxpool2x2(conv3)
        conv4 = cb("conv2d_8", cb("conv2d_7", pool3))
        drop4, c["keep4"] = drop(conv4, 1)
        pool4, c["pool4"] = maxpool2x2(drop4)
        cross = cb("conv2d_10", cb("conv2d_9", pool4))
        dropc, c["keepc"] = drop(cross, 2)
        up6 = tb("conv2d_transpose_1", dropc)
        conv6 = cb("conv2d_11", np.concatenate([drop4, up6], -1))
        up7 = tb("conv2d_transpose_2", conv6)
        conv7 = cb("conv2d_12", np.concatenate([conv3, up7], -1))
        up8 = tb("conv2d_transpose_3", conv7)
        conv8 = cb("conv2d_13", np.concatenate([conv2, up8], -1))
        up9 = tb("conv2d_transpose_4", conv8)
        conv9 = cb("conv2d_14", np.concatenate([conv1, up9], -1))
        z = conv2d_same(conv9, self.P["conv2d_15/kernel"], self.P["conv2d_15/bias"])
        yhat = sigmoid(z)
        c["head_x"] = conv9
        c["yhat"] = yhat
        c["shapes"] = dict(conv1=conv1.shape, conv2=conv2.shape, conv3=conv3.shape, drop4=drop4.shape)
        return yhat

    # ----- backward ------------------------------------------------------------
    def _convbn_bwd(self, name, dy, grads):
        c = self.cache[name]
        P = self.P
        bn = c["bn"]
        g = P[bn + "/gamma"]
        drs, dgs, dbs = [], [], []
        for dyy, rr, (m, v, _) in zip(np.split(dy, self.groups, 0), np.split(c["r"], self.groups, 0), c["stats"]):
            dr, dg, dbeta = bn_train_bwd(dyy, rr, g, m, v)
            drs.append(dr)
            dgs.append(dg)
            dbs.append(dbeta)
        dr = np.concatenate(drs, 0)
        grads[bn + "/gamma"] = np.sum(dgs, 0)
        grads[bn + "/beta"] = np.sum(dbs, 0)
        dz = self.q(dr * (c["r"] > 0))
        w = self.q(P[name + "/kernel"])
        if c["kind"] == "c3":
            dx, dw, db = conv2d_same_bwd(c["x"], w, dz, need_dx=(name != "conv2d_1"))
        else:
            dx, dw, db = tconv2x2s2_bwd(c["x"], w, dz)
        grads[name + "/kernel"] = dw
        grads[name + "/bias"] = db
        return None if dx is None else self.q(dx)

    def backward(self, target, valid_rows=None):
        """MSE loss on the last forward; returns (loss, acc, grads).  valid_rows: the loss and
        metric cover only output rows < valid_rows (U_net(pad=True)'s zero-padded frames:
        target [n, valid_rows, w, 3], padded rows get no loss gradient)."""
        c = self.cache
        t = np.asarray(target, self.dtype)
        yhat = c["yhat"]
        if valid_rows is not None:
            yv = yhat[:, :valid_rows]
            loss = mse(yv, t)
            acc = categorical_accuracy(t, yv)
            dz = np.zeros_like(yhat)
            dz[:, :valid_rows] = mse_grad_z(yv, t)
        else:
            loss = mse(yhat, t)
            acc = categorical_accuracy(t, yhat)
            dz = mse_grad_z(yhat, t)
        grads = {}
        dx9, dw, db = conv2d_same_bwd(c["head_x"], self.P["conv2d_15/kernel"], dz)
        grads["conv2d_15/kernel"] = dw
        grads["conv2d_15/bias"] = db
        s = c["shapes"]
        dm9 = self._convbn_bwd("conv2d_14", dx9, grads)
        c1 = s["conv1"][-1]
        dconv1, dup9 = dm9[..., :c1], dm9[..., c1:]
        dconv8 = self._convbn_bwd("conv2d_transpose_4", dup9, grads)
        dm8 = self._convbn_bwd("conv2d_13", dconv8, grads)
        c2 = s["conv2"][-1]
        dconv2, dup8 = dm8[..., :c2], dm8[..., c2:]
        dconv7 = self._convbn_bwd("conv2d_transpose_3", dup8, grads)
        dm7 = self._convbn_bwd("conv2d_12", dconv7, grads)
        c3 = s["conv3"][-1]
        dconv3, dup7 = dm7[..., :c3], dm7[..., c3:]
        dconv6 = self._convbn_bwd("conv2d_transpose_2", dup7, grads)
        dm6 = self._convbn_bwd("conv2d_11", dconv6, grads)
        c4 = s["drop4"][-1]
        ddrop4, dup6 = dm6[..., :c4], dm6[..., c4:]
        ddropc = self._convbn_bwd("conv2d_transpose_1", dup6, grads)
        dcross = ddropc * c["keepc"] * 2.0
        dpool4 = self._convbn_bwd("conv2d_9", self._convbn_bwd("conv2d_10", dcross, grads), grads)
        ddrop4 = ddrop4 + maxpool2x2_bwd(dpool4, c["pool4"], s["drop4"])
        dconv4 = ddrop4 * c["keep4"] * 2.0
        dpool3 = self._convbn_bwd("conv2d_7", self._convbn_bwd("conv2d_8", dconv4, grads), grads)
        dconv3 = dconv3 + maxpool2x2_bwd(dpool3, c["pool3"], s["conv3"])
        dpool2 = self._convbn_bwd("conv2d_5", self._convbn_bwd("conv2d_6", dconv3, grads), grads)
        dconv2 = dconv2 + maxpool2x2_bwd(dpool2, c["pool2"], s["conv2"])
        dpool1 = self._convbn_bwd("conv2d_3", self._convbn_bwd("conv2d_4", dconv2, grads), grads)
        dconv1 = dconv1 + maxpool2x2_bwd(dpool1, c["pool1"], s["conv1"])
        self._convbn_bwd("conv2d_1", self._convbn_bwd("conv2d_2", dconv1, grads), grads)
        return loss, acc, grads

    def apply_rmsprop(self, grads, accum):
        """One RMSprop step on trainables + BN moving-stat update (per group 0,
        i.e. what a single replica would hold)."""
        for k, gval in grads.items():
            a = accum.get(k, np.zeros_like(gval))
            self.P[k], accum[k] = rmsprop(self.P[k], gval, a)
        for name, entry in self.cache.items():
            if isinstance(entry, dict) and "stats" in entry and entry["stats"]:
                bn = entry["bn"]
                m, v, n = entry["stats"][0]
                mm, mv = bn_moving_update(self.P[bn + "/moving_mean"], self.P[bn + "/moving_variance"], m, v, n)
                self.P[bn + "/moving_mean"], self.P[bn + "/moving_variance"] = mm, mv
        return accum

    def train_step(self, x, t, accum, seed=0, groups=1):
        self.forward(x, training=True, seed=seed, groups=groups)
        loss, acc, grads = self.backward(t)
        self.apply_rmsprop(grads, accum)
        return loss, acc, grads


# --------------------------------------------------------------------------
# Config 1 (BASELINE.json configs[0]): 64x64 patch, 3-conv net, batch 1.
# conv3x3 3->32 + ReLU, conv3x3 32->32 + ReLU, conv1x1 32->3 + sigmoid.
# --------------------------------------------------------------------------
def init_tiny_params(seed=0, dtype=np.float64):
    rng = np.random.default_rng(seed)
    P = {}
    for name, ci, co, k in (("conv2d_1", 3, 32, 3), ("conv2d_2", 32, 32, 3)):
        std = np.sqrt(2.0 / (k * k * ci)) / 0.87962566103423978
        P[name + "/kernel"] = (truncated_normal(rng, (co, k, k, ci)) * std).astype(dtype)
        P[name + "/bias"] = np.zeros(co, dtype)
    lim = np.sqrt(6.0 / (32 + 3))
    P["conv2d_3/kernel"] = rng.uniform(-lim, lim, (3, 1, 1, 32)).astype(dtype)
    P["conv2d_3/bias"] = np.zeros(3, dtype)
    return P


class TinyNetRef:
    def __init__(self, params, dtype=np.float64):
        self.P = {k: np.asarray(v, dtype) for k, v in params.items()}
        self.dtype = dtype

    def forward(self, x):
        P = self.P
        x = np.asarray(x, self.dtype)
        z1 = conv2d_same(x, P["conv2d_1/kernel"], P["conv2d_1/bias"])
        r1 = np.maximum(z1, 0)
        z2 = conv2d_same(r1, P["conv2d_2/kernel"], P["conv2d_2/bias"])
        r2 = np.maximum(z2, 0)
        yhat = sigmoid(conv2d_same(r2, P["conv2d_3/kernel"], P["conv2d_3/bias"]))
        self.cache = dict(x=x, r1=r1, r2=r2, yhat=yhat)
        return yhat

    def backward(self, t):
        c, P = self.cache, self.P
        t = np.asarray(t, self.dtype)
        loss = mse(c["yhat"], t)
        g = {}
        dz3 = mse_grad_z(c["yhat"], t)
        dr2, g["conv2d_3/kernel"], g["conv2d_3/bias"] = conv2d_same_bwd(c["r2"], P["conv2d_3/kernel"], dz3)
        dz2 = dr2 * (c["r2"] > 0)
        dr1, g["conv2d_2/kernel"], g["conv2d_2/bias"] = conv2d_same_bwd(c["r1"], P["conv2d_2/kernel"], dz2)
        dz1 = dr1 * (c["r1"] > 0)
        _, g["conv2d_1/kernel"], g["conv2d_1/bias"] = conv2d_same_bwd(c["x"], P["conv2d_1/kernel"], dz1, need_dx=False)
        return loss, categorical_accuracy(t, c["yhat"]), g


# --------------------------------------------------------------------------
# predict() I/O conventions -- predict.py:59,64
# --------------------------------------------------------------------------
def png_to_input(u8):
    return np.true_divide(np.asarray(u8).astype(float), 255)


def output_to_png(pred):
    return (pred * 255).astype("uint8")  # truncation, predict.py:64
