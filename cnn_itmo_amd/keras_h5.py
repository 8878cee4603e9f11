"""Keras 2.2 HDF5 model files: ``save_model_hdf5`` / ``load_model_hdf5``.

The reference checkpoints the U-Net with ``ModelCheckpoint(...hdf5)``
(/root/reference/main.py:124, Keras ``Model.save``) and reloads it for
inference with ``keras.models.load_model('saved7-model-218-0.73.hdf5')``
(/root/reference/predict.py:24).  This module reads and writes the same file
layout, so a checkpoint trained with the reference loads here unchanged and a
checkpoint written here loads in Keras:

  /                     attrs keras_version, backend, model_config (JSON),
                              training_config (JSON)
  /model_weights        attrs layer_names, backend, keras_version
  /model_weights/<layer>            attrs weight_names ['<layer>/kernel:0', ...]
  /model_weights/<layer>/<layer>/kernel:0   dataset (Keras layout: Conv2D HWIO,
                                            Conv2DTranspose (kh, kw, Cout, Cin))
  /optimizer_weights    attrs weight_names; RMSprop accumulators, one per
                        trainable weight in model order (Keras 2.2.4
                        ``RMSprop.weights``; a leading ``iterations`` scalar,
                        as later Keras versions write, is accepted on load)

model_config is the Keras functional-API config ({"class_name": "Model",
"config": {"layers": [...], "input_layers", "output_layers"}}); every layer
class on the path maps to this package's layer of the same name.
"""
from __future__ import annotations

import json

import numpy as np

from . import hdf5
from .layers import (Activation, BatchNormalization, Concatenate, Conv2D, Conv2DTranspose, Dropout,
                     InputLayer, MaxPooling2D)

KERAS_VERSION = "2.2.4"
BACKEND = "tensorflow"

_INIT_CONFIGS = {
    "he_normal": {"class_name": "VarianceScaling",
                  "config": {"scale": 2.0, "mode": "fan_in", "distribution": "normal", "seed": None}},
    "glorot_uniform": {"class_name": "VarianceScaling",
                       "config": {"scale": 1.0, "mode": "fan_avg", "distribution": "uniform", "seed": None}},
    "zeros": {"class_name": "Zeros", "config": {}},
    "ones": {"class_name": "Ones", "config": {}},
}


def _init_config(name):
    if isinstance(name, dict):
        return name
    return _INIT_CONFIGS.get(name, {"class_name": str(name), "config": {}})


def _init_name(cfg):
    """Keras initializer config -> the string this package's initializers take."""
    if not isinstance(cfg, dict):
        return cfg
    c = cfg.get("config", {})
    cls = cfg.get("class_name", "")
    if cls == "VarianceScaling":
        key = (float(c.get("scale", 1.0)), c.get("mode"), c.get("distribution"))
        table = {(2.0, "fan_in", "normal"): "he_normal", (2.0, "fan_in", "truncated_normal"): "he_normal",
                 (1.0, "fan_avg", "uniform"): "glorot_uniform", (1.0, "fan_avg", "normal"): "glorot_normal"}
        return table.get(key, "glorot_uniform")
    return {"Zeros": "zeros", "Ones": "ones", "GlorotUniform": "glorot_uniform",
            "HeNormal": "he_normal"}.get(cls, "glorot_uniform")


def _null_regs():
    return {"kernel_regularizer": None, "bias_regularizer": None, "activity_regularizer": None,
            "kernel_constraint": None, "bias_constraint": None}


def layer_config(l):
    """Keras 2.2 ``layer.get_config()`` of one of this package's layers."""
    if isinstance(l, InputLayer):
        return {"batch_input_shape": [None] + list(l.shape), "dtype": "float32", "sparse": False, "name": l.name}
    base = {"name": l.name, "trainable": True}
    if isinstance(l, (Conv2D, Conv2DTranspose)):
        c = dict(base, filters=l.filters, kernel_size=list(l.kernel_size), strides=list(l.strides),
                 padding=l.padding, data_format="channels_last")
        if isinstance(l, Conv2D):
            c["dilation_rate"] = [1, 1]
        c.update(activation=l.activation or "linear", use_bias=l.use_bias,
                 kernel_initializer=_init_config(l.kernel_initializer),
                 bias_initializer=_init_config(getattr(l, "bias_initializer", "zeros")), **_null_regs())
        if isinstance(l, Conv2DTranspose):
            c["output_padding"] = None
        return c
    if isinstance(l, Activation):
        return dict(base, activation=l.activation)
    if isinstance(l, BatchNormalization):
        return dict(base, axis=-1, momentum=l.momentum, epsilon=l.epsilon, center=True, scale=True,
                    beta_initializer=_init_config("zeros"), gamma_initializer=_init_config("ones"),
                    moving_mean_initializer=_init_config("zeros"),
                    moving_variance_initializer=_init_config("ones"), beta_regularizer=None,
                    gamma_regularizer=None, beta_constraint=None, gamma_constraint=None)
    if isinstance(l, MaxPooling2D):
        return dict(base, pool_size=list(l.pool_size), padding="valid", strides=list(l.strides),
                    data_format="channels_last")
    if isinstance(l, Dropout):
        return dict(base, rate=l.rate, noise_shape=None, seed=None)
    if isinstance(l, Concatenate):
        return dict(base, axis=-1)
    raise NotImplementedError(type(l).__name__)


def model_config(model):
    layers = []
    for l in model.layers:
        inbound = [[[t.layer.name, 0, 0, {}] for t in l.inbound]] if l.inbound else []
        layers.append({"name": l.name, "class_name": l.type_name, "config": layer_config(l),
                       "inbound_nodes": inbound})
    return {"class_name": "Model",
            "config": {"name": model.name, "layers": layers,
                       "input_layers": [[model.inputs[0].layer.name, 0, 0]],
                       "output_layers": [[model.outputs[0].layer.name, 0, 0]]}}


def training_config(model):
    o = model.optimizer
    return {"optimizer_config": {"class_name": "RMSprop",
                                 "config": {"lr": o.lr, "rho": o.rho, "decay": 0.0, "epsilon": o.epsilon}},
            "loss": "mse", "metrics": ["accuracy"] if len(getattr(model, "metrics_names", [])) > 1 else [],
            "sample_weight_mode": None, "loss_weights": None}


def save_model_hdf5(model, path, include_optimizer=True, weights_only=False):
    """Keras ``Model.save`` / ``save_weights`` file layout (see module doc)."""
    from .model import _to_keras
    w = hdf5.Writer()
    named = model.named_weights()
    if not weights_only:
        w.attrs["keras_version"] = KERAS_VERSION
        w.attrs["backend"] = BACKEND
        w.attrs["model_config"] = json.dumps(model_config(model))
        mw = w.create_group("model_weights")
    else:
        mw = w.root
    mw.attrs["layer_names"] = [l.name for l in model.layers]
    mw.attrs["backend"] = BACKEND
    mw.attrs["keras_version"] = KERAS_VERSION
    trainable = []
    for l in model.layers:
        g = mw.create_group(l.name)
        names = []
        for wname, _, tr in l.weight_shapes():
            full = f"{l.name}/{wname}:0"
            names.append(full)
            g.create_dataset(full, _to_keras(l, wname, named[f"{l.name}/{wname}"]).astype(np.float32))
            if tr:
                trainable.append((l, wname))
        g.attrs["weight_names"] = names if names else np.zeros((0,), dtype="S1")
    if not weights_only and include_optimizer and model.optimizer is not None:
        w.attrs["training_config"] = json.dumps(training_config(model))
        accum = model.named_accumulators()
        if accum is not None:
            og = w.create_group("optimizer_weights")
            names = []
            for i, (l, wname) in enumerate(trainable):
                nm = "training/RMSprop/Variable%s:0" % ("" if i == 0 else f"_{i}")
                names.append(nm)
                og.create_dataset(nm, _to_keras(l, wname, accum[f"{l.name}/{wname}"]).astype(np.float32))
            og.attrs["weight_names"] = names
    w.save(path)


def _str(v):
    if isinstance(v, np.ndarray):
        v = v.item() if v.shape == () else v
    if isinstance(v, bytes):
        return v.decode("utf-8")
    return str(v)


def _str_list(v):
    if v is None:
        return []
    return [_str(x) for x in np.asarray(v, dtype=object).reshape(-1)]


def _attr_chunks(g, name):
    """Keras splits attributes over 64 KB into name0, name1, ... (save_attributes_to_hdf5_group)."""
    if name in g.attrs:
        return _str_list(g.attrs[name])
    out, i = [], 0
    while f"{name}{i}" in g.attrs:
        out += _str_list(g.attrs[f"{name}{i}"])
        i += 1
    return out


_CLASSES = {"InputLayer": InputLayer, "Conv2D": Conv2D, "Conv2DTranspose": Conv2DTranspose,
            "Activation": Activation, "BatchNormalization": BatchNormalization, "MaxPooling2D": MaxPooling2D,
            "Dropout": Dropout, "Concatenate": Concatenate}


def build_from_config(cfg, seed=0):
    """Rebuild a functional Model from a Keras model_config dict."""
    from .model import Model
    if cfg.get("class_name") not in ("Model", "Functional"):
        raise NotImplementedError(f"model class {cfg.get('class_name')!r} (functional models only)")
    c = cfg["config"]
    built = {}
    for node in c["layers"]:
        cls_name = node["class_name"]
        if cls_name not in _CLASSES:
            raise NotImplementedError(f"layer class {cls_name!r} is not on the CNN-ITMO path")
        lc = dict(node["config"])
        name = lc.pop("name", node.get("name"))
        if cls_name == "InputLayer":
            shp = lc.get("batch_input_shape") or lc.get("batch_shape")
            built[name] = InputLayer(tuple(shp[1:]), name=name).output
            continue
        for k in ("kernel_initializer", "bias_initializer"):
            if k in lc:
                lc[k] = _init_name(lc[k])
        if lc.get("data_format", "channels_last") != "channels_last":
            raise NotImplementedError("channels_first")
        layer = _CLASSES[cls_name](name=name, **{k: v for k, v in lc.items() if k != "trainable"})
        nodes = node.get("inbound_nodes") or []
        if len(nodes) != 1:
            raise NotImplementedError(f"{name}: shared layers / multiple inbound nodes")
        ins = []
        for ent in nodes[0]:
            src = ent["args"][0]["config"]["keras_history"][0] if isinstance(ent, dict) else ent[0]
            ins.append(built[src])
        built[name] = layer(ins if len(ins) > 1 else ins[0])
    inp = c["input_layers"][0][0]
    out = c["output_layers"][0][0]
    return Model(inputs=built[inp], outputs=built[out], name=c.get("name", "model_1"), seed=seed)


def _read_weights(model, g, by_name=False):
    """Keras 2.2 load_weights_from_hdf5_group: the file's layers with weights are
    matched to the model's layers with weights by POSITION (topological order; layer
    names may differ, e.g. when other models were built earlier in the session), the
    weights of a layer in order.  by_name=True (load_weights_from_hdf5_group_by_name):
    matched by layer name instead; file layers without a model layer of that name
    are skipped."""
    from .model import _to_internal
    names = _attr_chunks(g, "layer_names")
    named = {}
    with_w = [n for n in names if _attr_chunks(g[n], "weight_names")]
    if by_name:
        by = {l.name: l for l in model.layers if l.weight_shapes()}
        pairs = [(n, by[n]) for n in with_w if n in by]
    else:
        model_w = [l for l in model.layers if l.weight_shapes()]
        if len(with_w) != len(model_w):
            raise ValueError(f"You are trying to load a weight file containing {len(with_w)} layers into a "
                             f"model with {len(model_w)} layers.")
        pairs = list(zip(with_w, model_w))
    for fname, l in pairs:
        lg = g[fname]
        wn = _attr_chunks(lg, "weight_names")
        shapes = l.weight_shapes()
        if len(wn) != len(shapes):
            raise ValueError(f"Layer {l.name} expects {len(shapes)} weights, file has {len(wn)}")
        for nm, (wname, shp, _) in zip(wn, shapes):
            a = lg[nm].read()
            if tuple(a.shape) != tuple(shp):
                raise ValueError(f"{l.name}/{wname}: file shape {a.shape} != model shape {tuple(shp)}")
            named[f"{l.name}/{wname}"] = _to_internal(l, wname, np.asarray(a, np.float32))
    model.set_named_weights(named)


def load_weights_hdf5(model, path, by_name=False):
    f = hdf5.File(path)
    _read_weights(model, f["model_weights"] if "model_weights" in f else f.root, by_name=by_name)


def load_model_hdf5(path, compile=True):
    """keras.models.load_model for a Keras 2.2 HDF5 file (predict.py:24)."""
    from .model import RMSprop, _to_internal
    f = hdf5.File(path)
    if "model_config" not in f.attrs:
        raise ValueError("No model found in config file.")
    cfg = json.loads(_str(f.attrs["model_config"]))
    m = build_from_config(cfg)
    _read_weights(m, f["model_weights"])
    if compile and "training_config" in f.attrs:
        tc = json.loads(_str(f.attrs["training_config"]))
        oc = tc.get("optimizer_config", {})
        if oc.get("class_name", "RMSprop") != "RMSprop":
            raise NotImplementedError(f"optimizer {oc.get('class_name')!r}")
        o = oc.get("config", {})
        if float(o.get("decay", 0.0)):
            raise NotImplementedError("RMSprop decay is not on the path")
        m.compile(RMSprop(lr=o.get("lr", o.get("learning_rate", 1e-3)), rho=o.get("rho", 0.9),
                          epsilon=o.get("epsilon")), tc.get("loss", "mse"), tc.get("metrics") or ["accuracy"])
        if "optimizer_weights" in f:
            og = f["optimizer_weights"]
            wn = _attr_chunks(og, "weight_names")
            vals = [og[n].read() for n in wn]
            train = [(l, wname, shp) for l in m.layers for wname, shp, tr in l.weight_shapes() if tr]
            step = 0
            if len(vals) == len(train) + 1 and np.asarray(vals[0]).size == 1:
                step = int(np.asarray(vals[0]).reshape(-1)[0])  # iterations (later Keras versions)
                vals = vals[1:]
            if len(vals) == len(train):
                acc = {}
                for (l, wname, shp), v in zip(train, vals):
                    if tuple(v.shape) != tuple(shp):
                        raise ValueError(f"optimizer weight for {l.name}/{wname}: {v.shape} != {tuple(shp)}")
                    acc[f"{l.name}/{wname}"] = _to_internal(l, wname, np.asarray(v, np.float32))
                m._pending_accum = ("named", acc, step)
    return m
