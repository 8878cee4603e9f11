"""Reinhard tone mapping, the virtual camera and inverse Reinhard on the GPU
(SURVEY 8f row 4): the reference's dataset-generation and HDR-reconstruction
MATLAB scripts (m-files/Reinhard.m, virtual_camera.m, inverse_Reinhard.m),
float64 arithmetic in csrc/tonemap.hip behind the C ABI.

  reinhard(hdr)                -> SDR   (Reinhard.m:10-24: key 0.18 / log-average)
  virtual_camera(hdr, v, n, y) -> SDR   (virtual_camera.m:10-31: exposure 2^v,
                                         camera curve (1+n) X^y / (n + X^y), clipped at 1)
  virtual_camera_params(count, rng)     (v ~ U[-4, 4], n ~ N(0.6, 0.1), y ~ N(0.9, 0.1))
  inverse_reinhard(sdr_u8)     -> HDR   (inverse_Reinhard.m:1-23)
  crop(img, 284, 704)                   (imcrop(image, [704 284 511 511]): a 512 x 512 window)

Inputs: numpy arrays or CUDA tensors, NHWC RGB (HDR float32; SDR uint8).
Outputs: CUDA tensors (float32, or uint8 with ``out_u8=True``: imwrite's
``uint8(255*x)``).  ``RGB2Lum`` is called by the scripts but not part of the
reference; ``lum`` defaults to the Rec. 709 weights.

inverse_Reinhard.m as written reads ``ImgIn`` before assigning it; the only way
it runs is with ImgIn = the image being read.  ``mode='script'`` is that
script: uint8 SDR, 2.2 decode, X = I/(I-1) (whose sign makes every log term
realmin), G_E from the zero-luminance count, E clamped to [realmin, 2^32].
``mode='exact'`` is the algebraic inverse of Reinhard.m for a linear float SDR
image and a known HDR log-average ``g``: X = I/(1-I), E = g*X/a -- so
``inverse_reinhard(reinhard(hdr), g=log_average(hdr), mode='exact')``
reproduces ``hdr`` wherever L < 1.
"""
from __future__ import annotations

import ctypes

import numpy as np

REC709 = (0.2126, 0.7152, 0.0722)


def _dev(x, dtype):
    import torch
    t = torch.as_tensor(x)
    if t.dtype != dtype:
        t = t.to(dtype)
    t = t.cuda() if not t.is_cuda else t
    t = t.contiguous()
    if t.ndim == 3:
        t = t[None]
    if t.ndim != 4 or t.shape[-1] != 3:
        raise ValueError(f"expected NHWC RGB images, got shape {tuple(t.shape)}")
    return t


def _lum(lum):
    arr = (ctypes.c_double * 3)(*[float(c) for c in (lum or REC709)])
    return arr, ctypes.addressof(arr)


def _stats(mode, img, lum):
    import torch
    from . import ops
    from ._lib import call, query
    n, h, w, _ = img.shape
    ws = torch.empty(query("cnnitmo_tonemap_workspace_bytes", n), dtype=torch.uint8, device=img.device)
    stats = torch.empty(2 * n, dtype=torch.float64, device=img.device)
    keep, lp = _lum(lum)
    call("cnnitmo_tonemap_stats", mode, ops.ptr(img), n, h, w, lp, ops.ptr(stats), ops.ptr(ws), ws.numel(),
         ops.stream_ptr())
    del keep
    return stats


def log_average(hdr, lum=None):
    """exp(mean(log(max(Y, realmin)))) per image (the scripts' G), float64 [n]."""
    import torch
    img = _dev(hdr, torch.float32)
    st = _stats(0, img, lum)
    hw = img.shape[1] * img.shape[2]
    return torch.exp(st[0::2] * (1.0 / hw))


def _apply(curve, hdr, params, lum, out_u8):
    import torch
    from . import ops
    from ._lib import call
    img = _dev(hdr, torch.float32)
    n, h, w, _ = img.shape
    st = _stats(0, img, lum)
    p = torch.as_tensor(np.asarray(params, np.float64).reshape(n, 3)).cuda()
    out = torch.empty((n, h, w, 3), dtype=torch.uint8 if out_u8 else torch.float32, device=img.device)
    keep, lp = _lum(lum)
    call("cnnitmo_tonemap_apply", curve, ops.ptr(img), n, h, w, lp, ops.ptr(p), ops.ptr(st), 1 if out_u8 else 0,
         ops.ptr(out), ops.stream_ptr())
    del keep
    return out


def reinhard(hdr, key=0.18, lum=None, out_u8=False):
    """Reinhard.m: X = key/G * Y, L = X/(1+X), sdr = hdr * L/Y."""
    n = _dev(hdr, __import__("torch").float32).shape[0]
    return _apply(0, hdr, [[key, 0.0, 0.0]] * n, lum, out_u8)


def virtual_camera_params(count, rng=None):
    """virtual_camera.m:14,25-26 draws: v = 8*rand-4, n = normrnd(0.6, sqrt(0.1)),
    y = normrnd(0.9, sqrt(0.1)) (numpy's generator stands in for MATLAB's)."""
    rng = np.random.default_rng() if rng is None else rng
    v = 8 * rng.random(count) - 4
    cn = rng.normal(0.6, np.sqrt(0.1), count)
    cy = rng.normal(0.9, np.sqrt(0.1), count)
    return v, cn, cy


def virtual_camera(hdr, v, n, y, key=0.18, lum=None, out_u8=False):
    """virtual_camera.m: X = (key*2^v/G)*Y; X = min(1, (1+n) X^y/(n + X^y)); sdr = hdr * X/Y."""
    v, n, y = (np.atleast_1d(np.asarray(a, np.float64)) for a in (v, n, y))
    params = np.stack([key * 2.0 ** v, n, y], axis=1)
    return _apply(1, hdr, params, lum, out_u8)


def inverse_reinhard(sdr, a=0.18, lum=None, mode="script", g=1.0):
    """inverse_Reinhard.m (mode 'script': uint8 SDR in) or the exact inverse of
    Reinhard.m (mode 'exact': linear float SDR in, HDR log-average g) -> HDR fp32."""
    import torch
    from . import ops
    from ._lib import call
    if mode not in ("script", "exact"):
        raise ValueError(f"mode {mode!r}")
    img = _dev(sdr, torch.uint8 if mode == "script" else torch.float32)
    n, h, w, _ = img.shape
    st = _stats(1, img, lum) if mode == "script" else None
    out = torch.empty((n, h, w, 3), dtype=torch.float32, device=img.device)
    keep, lp = _lum(lum)
    call("cnnitmo_inverse_reinhard_apply", 1 if mode == "script" else 2, ops.ptr(img), n, h, w, lp,
         ops.ptr(st), float(a), float(g), ops.ptr(out), ops.stream_ptr())
    del keep
    return out


def crop(img, top=284, left=704, size=512):
    """imcrop(image, [left top size-1 size-1]) of Reinhard.m:10 (1-based MATLAB
    coordinates): rows top..top+size-1, columns left..left+size-1."""
    return img[..., top - 1:top - 1 + size, left - 1:left - 1 + size, :]
