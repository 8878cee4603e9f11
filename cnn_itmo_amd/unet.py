"""The CNN-ITMO network, built through the Keras-compatible layer API exactly as
/root/reference/model.py:195-289 wires it."""
from __future__ import annotations

from .layers import (BatchNormalization, Activation, Conv2D, Conv2DTranspose, Dropout, Input,
                     MaxPooling2D, concatenate)
from .model import Model


def ConvBN(filters, kernel_size, inputs):
    """Conv2D 'same' (he_normal) -> ReLU -> BatchNormalization  (model.py:195-196)."""
    return BatchNormalization()(Activation(activation="relu")(
        Conv2D(filters, kernel_size, padding="same", kernel_initializer="he_normal")(inputs)))


def ConvBNTranspose(filters, kernel_size, inputs):
    """Conv2DTranspose(strides=2, 'valid', he_normal) -> ReLU -> BN  (model.py:199-200)."""
    return BatchNormalization()(Activation(activation="relu")(
        Conv2DTranspose(filters, kernel_size, strides=2, padding="valid",
                        kernel_initializer="he_normal")(inputs)))


def U_net(pretrained_weights=None, input_size=(512, 512, 3), pad=False, dtype="float32", seed=0,
          verbose=True):
    """model.py:204-289.  ``pretrained_weights`` is accepted and ignored, as in the
    reference (its load is commented out at model.py:285-286).

    H and W must be divisible by 16 (4 pools, 4 x2 upsamplings, concat shape
    match) -- Keras itself raises a concat ValueError otherwise.  With
    ``pad=True`` H/W are rounded up to a multiple of 16 (1080p -> 1088) and
    ``predict`` zero-pads the input rows and crops the output."""
    h, w, c = input_size
    if pad:
        h, w = -(-h // 16) * 16, -(-w // 16) * 16
    if h % 16 or w % 16:
        raise ValueError(f"U_net input {input_size}: H and W must be multiples of 16 "
                         "(4 pooling levels + concatenation); pass pad=True to pad")
    inputs = Input((h, w, c))
    conv1 = ConvBN(32, 3, inputs)
    conv1 = ConvBN(32, 3, conv1)
    pool1 = MaxPooling2D(pool_size=(2, 2), strides=2)(conv1)
    conv2 = ConvBN(64, 3, pool1)
    conv2 = ConvBN(64, 3, conv2)
    pool2 = MaxPooling2D(pool_size=(2, 2), strides=2)(conv2)
    conv3 = ConvBN(128, 3, pool2)
    conv3 = ConvBN(128, 3, conv3)
    pool3 = MaxPooling2D(pool_size=(2, 2), strides=2)(conv3)
    conv4 = ConvBN(256, 3, pool3)
    conv4 = ConvBN(256, 3, conv4)
    drop4 = Dropout(0.5)(conv4)
    pool4 = MaxPooling2D(pool_size=(2, 2), strides=2)(drop4)
    conv_cross = ConvBN(512, 3, pool4)
    conv_cross = ConvBN(512, 3, conv_cross)
    drop_cross = Dropout(0.5)(conv_cross)
    up6 = ConvBNTranspose(512, 2, drop_cross)
    merge6 = concatenate([drop4, up6], axis=3)
    conv6 = ConvBN(512, 3, merge6)
    up7 = ConvBNTranspose(256, 2, conv6)
    merge7 = concatenate([conv3, up7], axis=3)
    conv7 = ConvBN(256, 3, merge7)
    up8 = ConvBNTranspose(128, 2, conv7)
    merge8 = concatenate([conv2, up8], axis=3)
    conv8 = ConvBN(128, 3, merge8)
    up9 = ConvBNTranspose(64, 2, conv8)
    merge9 = concatenate([conv1, up9], axis=3)
    conv9 = ConvBN(64, 3, merge9)
    OutImage = Conv2D(3, 1, activation="sigmoid")(conv9)
    model = Model(input=inputs, output=OutImage, name="ReinhardtPrediction", seed=seed)
    model.compile(optimizer="rmsprop", loss="mse", metrics=["accuracy"], dtype=dtype)
    if verbose:
        model.summary()
    return model


def TinyNet(input_size=(64, 64, 3), dtype="float32", seed=0):
    """BASELINE.json configs[0]: conv3x3 3->32 + ReLU, conv3x3 32->32 + ReLU,
    conv1x1 32->3 + sigmoid (a 3-conv plumbing net on 64x64 patches)."""
    inputs = Input(input_size)
    x = Conv2D(32, 3, padding="same", activation="relu", kernel_initializer="he_normal")(inputs)
    x = Conv2D(32, 3, padding="same", activation="relu", kernel_initializer="he_normal")(x)
    out = Conv2D(3, 1, activation="sigmoid")(x)
    model = Model(inputs=inputs, outputs=out, name="TinyNet", seed=seed)
    model.compile(optimizer="rmsprop", loss="mse", metrics=["accuracy"], dtype=dtype)
    return model
