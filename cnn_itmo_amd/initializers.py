"""Keras-2.2 weight initializers (distributions only; TF's RNG stream is not
reproducible outside TF, so initial weights are statistically -- not bitwise --
equal to the reference's).  he_normal: truncated normal, stddev
sqrt(2/fan_in)/0.8796 (Keras >= 2.2.3); glorot_uniform: U(+-sqrt(6/(fan_in+fan_out)));
fans from Keras' _compute_fans on the Keras kernel shape (kh, kw, in, out), which
for Conv2DTranspose's (kh, kw, Cout, Cin) kernel gives fan_in = 4*Cout."""
from __future__ import annotations

import numpy as np


def fans(keras_shape):
    rf = int(np.prod(keras_shape[:-2]))
    return keras_shape[-2] * rf, keras_shape[-1] * rf


def truncated_normal(rng, shape):
    """tf.truncated_normal(0, 1): values beyond 2 standard deviations are re-drawn
    (not clipped), so the distribution has no point masses and std 0.8796."""
    z = rng.standard_normal(shape)
    bad = np.abs(z) > 2.0
    while bad.any():
        z[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(z) > 2.0
    return z


def initialize(kind, keras_shape, rng):
    fan_in, fan_out = fans(keras_shape)
    if kind == "he_normal":
        std = np.sqrt(2.0 / fan_in) / 0.87962566103423978
        return truncated_normal(rng, keras_shape) * std
    if kind == "glorot_uniform":
        lim = np.sqrt(6.0 / (fan_in + fan_out))
        return rng.uniform(-lim, lim, keras_shape)
    if kind == "zeros":
        return np.zeros(keras_shape)
    if kind == "ones":
        return np.ones(keras_shape)
    raise ValueError(f"unsupported initializer {kind!r}")
