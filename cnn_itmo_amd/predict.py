"""Inference CLI with the reference's I/O conventions.

/root/reference/predict.py:24-70 loads a Keras checkpoint, then for every
``images_to_predict/input/*.png``: ``np.asarray(Image.open(f)).astype(float) / 255``
(float64, :59), ``model.predict`` on a batch of one (:62),
``(pred * 255)[0].astype('uint8')`` -- truncation, not rounding (:64) -- and
``Image.fromarray(...).save('images_to_predict/output/' + name)`` (:68-69).

Here the same conventions run batched on the GPU:

    python -m cnn_itmo_amd.predict --model saved7-model-218-0.73.hdf5 \\
        [--input images_to_predict/input] [--output images_to_predict/output] \\
        [--batch 8] [--dtype float32|bfloat16] [--tile TH,TW]

Differences, all deliberate: images are processed in sorted order, in batches
of equal-sized frames; the output file name is the input's base name (the
reference splits on a Windows '\\\\' separator, which on Linux yields the whole
input path); frames whose size differs from the checkpoint's input run
through a copy of the (fully convolutional) network built for their size,
padded to a multiple of 16 rows/columns and cropped back.
"""
from __future__ import annotations

import argparse
import glob
import os
import sys

import numpy as np


def read_png(path):
    """uint8 [H, W, 3] (grey / RGBA inputs are converted to RGB)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


def to_input(u8):
    """predict.py:59 -- float64 division by 255, then the model's float32."""
    return np.true_divide(np.asarray(u8).astype(float), 255).astype(np.float32)


def to_png(pred):
    """predict.py:64 -- (pred * 255).astype('uint8'): truncation toward zero."""
    return (np.asarray(pred, dtype=np.float32) * 255).astype("uint8")


def model_for_size(model, h, w, cache=None):
    """The same network and weights for frames of size (h, w): `model` itself when
    it fits (up to 15 rows short are padded by the engine), else a rebuilt copy
    whose input is (h, w) rounded up to multiples of 16."""
    H, W, _ = model.inputs[0].shape
    if W == w and 0 <= H - h < 16:
        return model
    key = (-(-h // 16) * 16, -(-w // 16) * 16)
    if cache is not None and key in cache:
        return cache[key]
    from . import keras_h5
    cfg = keras_h5.model_config(model)
    for node in cfg["config"]["layers"]:
        if node["class_name"] == "InputLayer":
            node["config"]["batch_input_shape"] = [None, key[0], key[1], 3]
    m = keras_h5.build_from_config(cfg)
    m.set_named_weights(model.named_weights())
    m.compile(optimizer="rmsprop", loss="mse", metrics=["accuracy"], dtype=model.dtype)
    if cache is not None:
        cache[key] = m
    return m


def _pad_cols(x, W):
    if x.shape[2] == W:
        return x
    out = np.zeros(x.shape[:2] + (W, x.shape[3]), dtype=x.dtype)
    out[:, :, :x.shape[2]] = x
    return out


def predict_frames(model, frames_u8, batch=8, cache=None, tile=None):
    """uint8 frames (equal sizes) -> uint8 predictions, reference conventions.
    ``tile`` (th, tw): spatially tiled inference with 96-px halos (tiled.py; same
    result, activation memory bounded by the window instead of the frame)."""
    h, w = frames_u8[0].shape[:2]
    if tile is not None:
        from .tiled import predict_tiled
        outs = []
        for i in range(0, len(frames_u8), batch):
            x = np.stack([to_input(f) for f in frames_u8[i:i + batch]])
            y = predict_tiled(model, x, tile, batch_size=batch, cache=cache)
            outs.extend(to_png(y[j]) for j in range(y.shape[0]))
        return outs
    m = model_for_size(model, h, w, cache)
    W = m.inputs[0].shape[1]
    outs = []
    for i in range(0, len(frames_u8), batch):
        x = np.stack([to_input(f) for f in frames_u8[i:i + batch]])
        y = m.predict(_pad_cols(x, W), batch_size=batch)
        outs.extend(to_png(y[j, :h, :w]) for j in range(y.shape[0]))
    return outs


def predict_dir(model, in_dir, out_dir, batch=8, pattern="*.png", log=print, tile=None):
    from PIL import Image
    files = sorted(glob.glob(os.path.join(in_dir, pattern)))
    if not files:
        raise FileNotFoundError(f"no {pattern} files in {in_dir}")
    os.makedirs(out_dir, exist_ok=True)
    groups = {}
    frames = {f: read_png(f) for f in files}
    for f in files:
        groups.setdefault(frames[f].shape, []).append(f)
    cache = {}
    written = []
    for shape, fs in groups.items():
        log(f"Grabbing {len(fs)} input files of {shape[1]}x{shape[0]}")
        preds = predict_frames(model, [frames[f] for f in fs], batch, cache, tile)
        for f, p in zip(fs, preds):
            dst = os.path.join(out_dir, os.path.basename(f))
            Image.fromarray(p).save(dst)
            written.append(dst)
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", required=True, help="Keras HDF5 checkpoint (or an .npz from Model.save)")
    ap.add_argument("--input", default="images_to_predict/input")
    ap.add_argument("--output", default="images_to_predict/output")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--tile", default=None, help="TH,TW: spatially tiled inference (multiples of 16; 96-px halos)")
    a = ap.parse_args(argv)
    tile = tuple(int(v) for v in a.tile.split(",")) if a.tile else None
    from .model import load_model
    m = load_model(a.model)
    if m.optimizer is None:
        m.compile(optimizer="rmsprop", loss="mse", metrics=["accuracy"])
    m.set_dtype(a.dtype)
    out = predict_dir(m, a.input, a.output, a.batch, tile=tile)
    print(f"wrote {len(out)} predictions to {a.output}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
