"""Keras-2.2-compatible functional layer API (the reference's operator boundary).

The reference builds its network with ``keras.layers`` calls
(/root/reference/model.py:195-278): ``Input``, ``Conv2D``, ``Conv2DTranspose``,
``Activation``, ``BatchNormalization``, ``MaxPooling2D``, ``Dropout`` and
``concatenate``.  The same calls here build a symbolic graph; ``Model``
(model.py) compiles it into fused HIP-kernel stages (engine.py).  Names,
argument meaning, output shapes, parameter counts and build-time ValueErrors
follow Keras 2.2 so ``summary()`` reproduces /root/reference/layers.txt.
"""
from __future__ import annotations

import collections
import itertools

_name_counts: collections.Counter = collections.Counter()
_seq = itertools.count()


def clear_session():
    """Reset automatic layer naming (keras.backend.clear_session)."""
    _name_counts.clear()


def _auto_name(prefix):
    _name_counts[prefix] += 1
    return f"{prefix}_{_name_counts[prefix]}"


def _pair(v):
    if isinstance(v, int):
        return (v, v)
    v = tuple(v)
    if len(v) != 2:
        raise ValueError(f"expected an int or a pair, got {v!r}")
    return v


class KTensor:
    """Symbolic NHWC tensor; ``shape`` excludes the batch dimension."""

    def __init__(self, shape, layer, inputs):
        self.shape = tuple(shape)
        self.layer = layer
        self.inputs = list(inputs)

    def __repr__(self):
        return f"<KTensor {self.layer.name} shape=(None, {', '.join(map(str, self.shape))})>"


class Layer:
    prefix = "layer"
    type_name = "Layer"

    def __init__(self, name=None, **kwargs):
        self.name = name or _auto_name(self.prefix)
        self.inbound = []
        self.output = None
        self.seq = None

    # ---- Keras-style call ------------------------------------------------
    def __call__(self, inputs):
        xs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        for t in xs:
            if not isinstance(t, KTensor):
                raise ValueError(f"Layer {self.name} was called with a non-symbolic input {t!r}")
        if self.output is not None:
            raise ValueError(f"Layer {self.name} is already connected (shared layers are not supported)")
        shape = self.compute_output_shape([t.shape for t in xs])
        self.inbound = xs
        self.seq = next(_seq)
        self.output = KTensor(shape, self, xs)
        return self.output

    def compute_output_shape(self, shapes):
        raise NotImplementedError

    def weight_shapes(self):
        """[(name, shape, trainable)] in Keras order."""
        return []

    def count_params(self):
        n = 0
        for _, s, _ in self.weight_shapes():
            k = 1
            for d in s:
                k *= d
            n += k
        return n

    def get_config(self):
        return {"name": self.name}


class InputLayer(Layer):
    prefix = "input"
    type_name = "InputLayer"

    def __init__(self, shape, name=None):
        super().__init__(name)
        self.shape = tuple(shape)
        if len(self.shape) != 3:
            raise ValueError(f"Input shape must be (H, W, C), got {shape!r}")
        self.seq = next(_seq)
        self.output = KTensor(self.shape, self, [])

    def get_config(self):
        return {"name": self.name, "shape": list(self.shape)}


def Input(shape=None, name=None, **kwargs):
    """keras.layers.Input (model.py:207)."""
    if shape is None:
        shape = kwargs.get("batch_shape", (None,) * 4)[1:]
    return InputLayer(shape, name).output


_ACTS = (None, "linear", "relu", "sigmoid")


class Conv2D(Layer):
    """keras.layers.Conv2D -- 'same'/'valid', stride 1, TF cross-correlation (model.py:196,276)."""

    prefix = "conv2d"
    type_name = "Conv2D"

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 name=None, **kwargs):
        super().__init__(name)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        if activation not in _ACTS:
            raise ValueError(f"Unsupported activation {activation!r}")
        self.activation = None if activation == "linear" else activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer
        if self.strides != (1, 1):
            raise NotImplementedError("Conv2D strides != 1 are not on the CNN-ITMO path")
        if self.padding not in ("same", "valid"):
            raise ValueError(f"Invalid padding {padding!r}")

    def compute_output_shape(self, shapes):
        if len(shapes) != 1:
            raise ValueError("Conv2D takes one input")
        h, w, c = shapes[0]
        self.in_channels = c
        kh, kw = self.kernel_size
        if self.padding == "valid":
            h, w = h - kh + 1, w - kw + 1
            if h <= 0 or w <= 0:
                raise ValueError(f"Negative dimension size in {self.name}")
        return (h, w, self.filters)

    def weight_shapes(self):
        kh, kw = self.kernel_size
        ws = [("kernel", (kh, kw, self.in_channels, self.filters), True)]
        if self.use_bias:
            ws.append(("bias", (self.filters,), True))
        return ws

    def get_config(self):
        return {"name": self.name, "filters": self.filters, "kernel_size": list(self.kernel_size),
                "padding": self.padding, "activation": self.activation, "use_bias": self.use_bias,
                "kernel_initializer": self.kernel_initializer}


class Conv2DTranspose(Layer):
    """keras.layers.Conv2DTranspose -- 2x2 stride-2 'valid' upsampling (model.py:200)."""

    prefix = "conv2d_transpose"
    type_name = "Conv2DTranspose"

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None,
                 use_bias=True, kernel_initializer="glorot_uniform", bias_initializer="zeros",
                 name=None, **kwargs):
        super().__init__(name)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        if activation not in _ACTS:
            raise ValueError(f"Unsupported activation {activation!r}")
        self.activation = None if activation == "linear" else activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        if self.kernel_size != (2, 2) or self.strides != (2, 2) or self.padding != "valid":
            raise NotImplementedError("only Conv2DTranspose(f, 2, strides=2, padding='valid') is on the path")

    def compute_output_shape(self, shapes):
        h, w, c = shapes[0]
        self.in_channels = c
        return (2 * h, 2 * w, self.filters)

    def weight_shapes(self):
        ws = [("kernel", (2, 2, self.filters, self.in_channels), True)]
        if self.use_bias:
            ws.append(("bias", (self.filters,), True))
        return ws

    def get_config(self):
        return {"name": self.name, "filters": self.filters, "kernel_size": list(self.kernel_size),
                "strides": list(self.strides), "padding": self.padding, "activation": self.activation,
                "kernel_initializer": self.kernel_initializer}


class Activation(Layer):
    prefix = "activation"
    type_name = "Activation"

    def __init__(self, activation, name=None, **kwargs):
        super().__init__(name)
        if activation not in ("relu", "sigmoid", "linear"):
            raise ValueError(f"Unsupported activation {activation!r}")
        self.activation = activation

    def compute_output_shape(self, shapes):
        return shapes[0]

    def get_config(self):
        return {"name": self.name, "activation": self.activation}


class BatchNormalization(Layer):
    """keras.layers.BatchNormalization (axis=-1, momentum=0.99, epsilon=1e-3)."""

    prefix = "batch_normalization"
    type_name = "BatchNormalization"

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, name=None,
                 **kwargs):
        super().__init__(name)
        if axis not in (-1, 3):
            raise NotImplementedError("BatchNormalization only on the channel axis")
        if not (center and scale):
            raise NotImplementedError("center=False/scale=False are not on the path")
        self.momentum = float(momentum)
        self.epsilon = float(epsilon)

    def compute_output_shape(self, shapes):
        self.channels = shapes[0][-1]
        return shapes[0]

    def weight_shapes(self):
        c = self.channels
        return [("gamma", (c,), True), ("beta", (c,), True), ("moving_mean", (c,), False),
                ("moving_variance", (c,), False)]

    def get_config(self):
        return {"name": self.name, "momentum": self.momentum, "epsilon": self.epsilon}


class MaxPooling2D(Layer):
    prefix = "max_pooling2d"
    type_name = "MaxPooling2D"

    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None, **kwargs):
        super().__init__(name)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        if self.pool_size != (2, 2) or self.strides != (2, 2) or padding != "valid":
            raise NotImplementedError("only MaxPooling2D((2,2), strides=2, 'valid') is on the path")

    def compute_output_shape(self, shapes):
        h, w, c = shapes[0]
        return (h // 2, w // 2, c)

    def get_config(self):
        return {"name": self.name, "pool_size": list(self.pool_size)}


class Dropout(Layer):
    prefix = "dropout"
    type_name = "Dropout"

    def __init__(self, rate, name=None, **kwargs):
        super().__init__(name)
        self.rate = float(rate)
        if self.rate != 0.5:
            raise NotImplementedError("Dropout rate 0.5 is the one on the path (model.py:226,239)")

    def compute_output_shape(self, shapes):
        return shapes[0]

    def get_config(self):
        return {"name": self.name, "rate": self.rate}


class Concatenate(Layer):
    prefix = "concatenate"
    type_name = "Concatenate"

    def __init__(self, axis=-1, name=None, **kwargs):
        super().__init__(name)
        if axis not in (-1, 3):
            raise NotImplementedError("concatenate only on the channel axis")

    def compute_output_shape(self, shapes):
        if len(shapes) < 2:
            raise ValueError("A `Concatenate` layer should be called on a list of at least 2 inputs")
        h, w = shapes[0][:2]
        for s in shapes[1:]:
            if tuple(s[:2]) != (h, w):
                raise ValueError("A `Concatenate` layer requires inputs with matching shapes except "
                                 f"for the concat axis. Got inputs shapes: {[(None,) + tuple(x) for x in shapes]}")
        return (h, w, sum(s[2] for s in shapes))


def concatenate(inputs, axis=-1, **kwargs):
    """keras.layers.concatenate (model.py:246,251,256,261)."""
    return Concatenate(axis=axis, **kwargs)(inputs)


LAYER_CLASSES = {c.type_name: c for c in (InputLayer, Conv2D, Conv2DTranspose, Activation,
                                          BatchNormalization, MaxPooling2D, Dropout, Concatenate)}
