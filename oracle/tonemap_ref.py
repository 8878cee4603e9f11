"""CPU oracle for the tone-mapping maps -- TEST INFRASTRUCTURE ONLY.

numpy float64 restatement of the reference's MATLAB scripts, line for line:
  Reinhard.m:10-24        (log-average G over the crop, X = 0.18/G * Y, L = X/(1+X))
  virtual_camera.m:10-31  (delta_t = 0.18*2^v/G, (1+n) X^y / (n + X^y), min(1, .))
  inverse_Reinhard.m:1-23 (In = (u8/255)^2.2, X = I/(I-1) [or I/(1-I)], G_E, E clamps)
The scripts' luminance function RGB2Lum is not in the reference (parity
unpinned for it; the weights are a parameter).  The scripts' log sums are
sequential loops (`sum = sum + log(...)` over rows, then columns): np.cumsum
reproduces that order.  MATLAB's min(1, NaN) is 1 (np.fmin); its uint8()
rounds half away from zero and saturates, NaN -> 0.
"""
import numpy as np

REALMIN = np.finfo(np.float64).tiny
REC709 = (0.2126, 0.7152, 0.0722)


def rgb2lum(img, lum=REC709):
    img = np.asarray(img, np.float64)
    return lum[0] * img[..., 0] + lum[1] * img[..., 1] + lum[2] * img[..., 2]


def seq_sum(a):
    a = np.asarray(a, np.float64).reshape(-1)
    return float(np.cumsum(a)[-1]) if a.size else 0.0


def log_average(Y):
    return np.exp(seq_sum(np.log(np.maximum(Y, REALMIN))) * (1.0 / Y.size))


def reinhard(hdr, key=0.18, lum=REC709):
    """One image [H, W, 3] -> float64 SDR (before imwrite)."""
    Y = rgb2lum(hdr, lum)
    with np.errstate(divide="ignore", invalid="ignore"):
        G = log_average(Y)
        X = (key / G) * Y
        L = X / (1 + X)
        return np.asarray(hdr, np.float64) * (L / Y)[..., None]


def virtual_camera(hdr, v, n, y, key=0.18, lum=REC709):
    Y = rgb2lum(hdr, lum)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        G = log_average(Y)
        X = (key * 2.0 ** v / G) * Y
        Xy = X ** y
        X = np.fmin(1.0, (1 + n) * (Xy / (n + Xy)))
        return np.asarray(hdr, np.float64) * (X / Y)[..., None]


def inverse_reinhard(sdr, a=0.18, lum=REC709, mode="script", g=1.0):
    """mode 'script': inverse_Reinhard.m (uint8 in, ImgIn := the image); mode
    'exact': linear float SDR in, E = g*X/a with X = I/(1-I)."""
    if mode == "script":
        In = (np.asarray(sdr, np.float64) / 255) ** 2.2
    else:
        In = np.asarray(sdr, np.float64)
    I = rgb2lum(In, lum)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        if mode == "script":
            X = I / (I - 1)
            GX = np.exp(seq_sum(np.log(np.maximum(X, REALMIN))) * (1.0 / I.size))
            P = float(I.size)
            PB1 = float(np.count_nonzero(I == 0))
            PB2 = float(np.count_nonzero(I != 0))
            GE = np.exp(P * np.log(GX) / PB1 - PB2 * np.log(a) / PB1)
        else:
            X = I / (1 - I)
            GE = g
        E = GE * X / a
        E[np.isnan(E)] = REALMIN
        E[E >= 2.0 ** 32] = 2.0 ** 32
        return In * (E / I)[..., None]


def im2uint8(x):
    """MATLAB uint8(255*x) as imwrite applies it to doubles."""
    v = 255.0 * np.asarray(x, np.float64)
    out = np.zeros(v.shape, np.uint8)
    ok = v > 0
    out[ok] = np.minimum(np.floor(v[ok] + 0.5), 255).astype(np.uint8)
    return out
