"""cnn_itmo_amd -- MI355X-native (gfx950) CNN-ITMO SDR->HDR U-Net hot path.

Keras-compatible front end (layers, Model, U_net, ConvBN, ConvBNTranspose,
load_model) over hand-written HIP kernels in lib/libcnnitmo.so (C ABI:
include/cnn_itmo.h).  No CPU fallback: the engine raises without a ROCm GPU.
"""
from .layers import (Activation, BatchNormalization, Concatenate, Conv2D, Conv2DTranspose, Dropout,
                     Input, InputLayer, MaxPooling2D, clear_session, concatenate)
from .model import Model, RMSprop, load_model
from .unet import ConvBN, ConvBNTranspose, TinyNet, U_net
from .callbacks import CSVLogger, LambdaCallback, ModelCheckpoint

__all__ = ["Activation", "BatchNormalization", "Concatenate", "Conv2D", "Conv2DTranspose", "Dropout",
           "Input", "InputLayer", "MaxPooling2D", "clear_session", "concatenate", "Model", "RMSprop",
           "load_model", "ConvBN", "ConvBNTranspose", "TinyNet", "U_net", "CSVLogger",
           "LambdaCallback", "ModelCheckpoint"]
