"""keras.models.Model-compatible wrapper around the HIP engine.

Covers the model API the reference uses:
``Model(input=, output=, name=)`` (model.py:278), ``compile('rmsprop', 'mse',
['accuracy'])`` (:281), ``summary()`` (:288, output == layers.txt),
``predict(X)`` (predict.py:62), ``fit_generator(...)`` (main.py:126-132),
``train_on_batch``, ``evaluate``, ``save`` / ``load_model`` (predict.py:24,
main.py:124) plus ``get_weights``/``set_weights`` in Keras layouts.

Data parallelism sits behind the same calls: under torchrun (one
process per GPU, ``dist.init_from_env()``), ``fit_generator(...,
distributed=True)`` -- or any training call after ``model.distribute()`` --
shards the batch stream per rank (each rank's generator yields its own batch;
``flow_from_directory`` shards itself), all-reduces the gradients with RCCL
during backward and averages the BN moving statistics (``dist.py``).  Epoch
logs are global (all ranks' batches, weighted by size); callbacks run on rank 0.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

from . import initializers
from .layers import (LAYER_CLASSES, BatchNormalization, Conv2D, Conv2DTranspose, InputLayer, KTensor,
                     Layer)


class RMSprop:
    """keras.optimizers.RMSprop(lr=0.001, rho=0.9, epsilon=None->1e-7, decay=0)."""

    def __init__(self, lr=0.001, rho=0.9, epsilon=None, decay=0.0, **kwargs):
        self.lr = float(kwargs.get("learning_rate", lr))
        self.rho = float(rho)
        self.epsilon = 1e-7 if epsilon is None else float(epsilon)
        if decay:
            raise NotImplementedError("RMSprop decay is not on the path")


def _to_internal(layer, wname, arr):
    """Keras layout -> engine layout (Conv2D kernel HWIO -> OHWI)."""
    if isinstance(layer, Conv2D) and wname == "kernel":
        return np.ascontiguousarray(np.transpose(arr, (3, 0, 1, 2)))
    return arr


def _to_keras(layer, wname, arr):
    if isinstance(layer, Conv2D) and wname == "kernel":
        return np.ascontiguousarray(np.transpose(arr, (1, 2, 3, 0)))
    return arr


class History:
    def __init__(self):
        self.epoch = []
        self.history = {}


class Model:
    def __init__(self, inputs=None, outputs=None, name=None, **kwargs):
        inputs = kwargs.pop("input", inputs)
        outputs = kwargs.pop("output", outputs)
        self.inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        self.outputs = list(outputs) if isinstance(outputs, (list, tuple)) else [outputs]
        if len(self.inputs) != 1 or len(self.outputs) != 1:
            raise NotImplementedError("single-input single-output models only")
        self.name = name or "model_1"
        # collect layers reachable from the output, in creation order
        seen, stack = {}, [self.outputs[0]]
        while stack:
            t = stack.pop()
            if id(t.layer) in seen:
                continue
            seen[id(t.layer)] = t.layer
            stack.extend(t.inputs)
        if id(self.inputs[0].layer) not in seen:
            raise ValueError("the output is not connected to the input")
        self.layers = sorted(seen.values(), key=lambda l: l.seq)
        self._weights = {}  # internal-layout numpy weights (host copy, authoritative before engine)
        self.optimizer = None
        self.engine = None
        self._dp = None          # dist.GradBucketer once distribute() was called
        self._dp_args = None
        self.dtype = "float32"
        self.stop_training = False
        self._init_weights(kwargs.get("seed", 0))

    # ---- weights -------------------------------------------------------------
    def _init_weights(self, seed):
        rng = np.random.default_rng(seed)
        for l in self.layers:
            for wname, shp, _ in l.weight_shapes():
                if isinstance(l, BatchNormalization):
                    v = np.ones(shp) if wname in ("gamma", "moving_variance") else np.zeros(shp)
                elif wname == "bias":
                    v = np.zeros(shp)
                else:
                    v = initializers.initialize(getattr(l, "kernel_initializer", "glorot_uniform"), shp, rng)
                self._weights[f"{l.name}/{wname}"] = _to_internal(l, wname, v).astype(np.float32)

    def named_weights(self):
        """Internal-layout weights keyed 'layer/weight' (engine copy if live)."""
        if self.engine is not None:
            self._weights.update(self.engine.get_weights())
        return {k: v.copy() for k, v in self._weights.items()}

    def set_named_weights(self, named):
        for k, v in named.items():
            if k not in self._weights:
                raise KeyError(k)
            if tuple(np.shape(v)) != self._weights[k].shape:
                raise ValueError(f"{k}: shape {np.shape(v)} != {self._weights[k].shape}")
            self._weights[k] = np.asarray(v, np.float32).copy()
        if self.engine is not None:
            self.engine.set_weights({k: self._weights[k] for k in named})

    def get_weights(self):
        """Keras order and layouts (Conv2D kernels HWIO)."""
        named = self.named_weights()
        out = []
        for l in self.layers:
            for wname, _, _ in l.weight_shapes():
                out.append(_to_keras(l, wname, named[f"{l.name}/{wname}"]))
        return out

    def set_weights(self, weights):
        it = iter(weights)
        named = {}
        for l in self.layers:
            for wname, shp, _ in l.weight_shapes():
                w = np.asarray(next(it))
                if tuple(w.shape) != tuple(shp):
                    raise ValueError(f"{l.name}/{wname}: expected {shp}, got {w.shape}")
                named[f"{l.name}/{wname}"] = _to_internal(l, wname, w)
        self.set_named_weights(named)

    def count_params(self):
        return sum(l.count_params() for l in self.layers)

    # ---- compile / engine ------------------------------------------------------
    def compile(self, optimizer="rmsprop", loss="mse", metrics=None, dtype=None, **kwargs):
        if isinstance(optimizer, str):
            if optimizer.lower() != "rmsprop":
                raise NotImplementedError(f"optimizer {optimizer!r} (only 'rmsprop' is on the path)")
            optimizer = RMSprop()
        if loss not in ("mse", "mean_squared_error"):
            raise NotImplementedError(f"loss {loss!r} (only 'mse' is on the path)")
        for m in metrics or []:
            if m not in ("accuracy", "acc", "categorical_accuracy"):
                raise NotImplementedError(f"metric {m!r}")
        self.optimizer = optimizer
        self.metrics_names = ["loss"] + (["acc"] if metrics else [])
        if dtype is not None:
            self.set_dtype(dtype)

    def set_dtype(self, dtype):
        if dtype not in ("float32", "bfloat16"):
            raise ValueError("dtype must be 'float32' or 'bfloat16'")
        if dtype != self.dtype and self.engine is not None:
            self._weights.update(self.engine.get_weights())
            acc = self.engine.accum.clone()
            step = self.engine.step
            self.engine = None
            self.dtype = dtype
            self._engine()
            self.engine.accum.copy_(acc)
            self.engine.step = step  # the default dropout seed continues (no repeated masks)
        self.dtype = dtype

    def _engine(self):
        if self.engine is None:
            from .engine import Engine
            self.engine = Engine(self, dtype=self.dtype)
            self.engine.set_weights(self._weights)
            pending = getattr(self, "_pending_accum", None)
            if pending is not None:
                import torch
                if isinstance(pending[0], str):  # ("named", {key: array}, step): per-tensor accumulators (Keras HDF5 optimizer_weights)
                    for k, v in pending[1].items():
                        off, shp = self.engine.pslices[k]
                        self.engine.accum[off:off + int(np.prod(shp))].copy_(
                            torch.as_tensor(np.ascontiguousarray(v, np.float32).reshape(-1)))
                    self.engine.step = pending[2]
                else:
                    self.engine.accum.copy_(torch.as_tensor(pending[0]))
                    self.engine.step = pending[1]
                self._pending_accum = None
            if self._dp_args is not None:  # re-wire DP into a rebuilt engine (dtype switch)
                from . import dist as D
                self._dp = D.attach(self.engine, *self._dp_args, broadcast=False)
        return self.engine

    # ---- data parallelism ----------------------------------------------------------
    def distribute(self, bucket_mb=16.0, group=None):
        """Train this model data-parallel over the initialised torch.distributed group
        (one process per GPU; backend ``nccl`` = RCCL).  Rank 0's weights, moving stats
        and optimizer state are broadcast first (DDP semantics).  Returns self."""
        import torch.distributed as tdist
        if not (tdist.is_available() and tdist.is_initialized()):
            raise RuntimeError("distribute() needs an initialised process group (cnn_itmo_amd.dist.init_from_env)")
        if self._dp is None:
            from . import dist as D
            self._dp_args = (float(bucket_mb), group)
            self._dp = D.attach(self._engine(), bucket_mb, group)
        return self

    @property
    def world(self):
        """(rank, world) this model trains over (0, 1) when not distributed."""
        if self._dp is None:
            return 0, 1
        from . import dist as D
        return D.rank_world(self._dp_args[1])

    def _allreduce_sum(self, vals):
        """Sum a small host vector over the DP ranks (identity when not distributed)."""
        if self._dp is None or self._dp.world == 1:
            return np.asarray(vals, np.float64)
        import torch
        import torch.distributed as tdist
        t = torch.tensor(np.asarray(vals, np.float64), device=self.engine.grads.device)
        tdist.all_reduce(t, group=self._dp_args[1])
        return t.cpu().numpy()

    @property
    def input_shape(self):
        return (None,) + self.inputs[0].shape

    # ---- inference -------------------------------------------------------------
    def _to_dev(self, x):
        """Host arrays are copied in; CUDA tensors (e.g. datagen batches) are used as they are."""
        import torch
        if isinstance(x, torch.Tensor):
            return x.float().cuda() if not x.is_cuda else x.float()
        return torch.as_tensor(np.asarray(x, dtype=np.float32)).cuda()

    def predict(self, x, batch_size=32, verbose=0, steps=None):
        """model.predict (predict.py:62): x [N,H,W,3] float -> float32 [N,H,W,3].
        H may be up to 15 rows short of the model height (zero-padded, output cropped)."""
        eng = self._engine()
        x = np.asarray(x)
        if x.ndim != 4:
            raise ValueError(f"expected a 4-D NHWC batch, got shape {x.shape}")
        outs = []
        for i in range(0, x.shape[0], batch_size):
            outs.append(eng.predict(self._to_dev(x[i:i + batch_size])).cpu().numpy())
        return np.concatenate(outs, 0)

    # ---- training ----------------------------------------------------------------
    def _check_compiled(self):
        if self.optimizer is None:
            raise RuntimeError("You must compile your model before using it.")

    def train_on_batch(self, x, y, sync=True, global_batch=None):
        """One step on this rank's batch.  Distributed: every rank applies the same update,
        the gradient of the GLOBAL batch mean when ``global_batch`` (the frames over all
        ranks) is given -- each rank's loss gradient is normalised by global_batch/world
        frames, so unequal shares are weighted by their size -- and otherwise the mean of
        the ranks' batch-mean gradients.  The returned loss/acc are this rank's."""
        self._check_compiled()
        if len(x) == 0:
            raise ValueError("train_on_batch: empty batch (a data-parallel rank got no frames of a global batch "
                             "smaller than the world size; such batches must be dropped on every rank)")
        eng = self._engine()
        o = self.optimizer
        kw = {}
        if self._dp is not None:
            r, w = self.world
            # per-rank dropout masks: seed = step*world + rank (one stream per replica)
            kw = dict(sync=self._dp.finish, grad_scale=self._dp.grad_scale, seed=eng.step * w + r)
            if global_batch is not None:
                kw["grad_frames"] = float(global_batch) / w
        la = eng.train_step(self._to_dev(x), self._to_dev(y), lr=o.lr, rho=o.rho, eps=o.epsilon, **kw)
        return la.cpu().numpy().tolist() if sync else la

    def evaluate(self, x, y, batch_size=32, verbose=0):
        self._check_compiled()
        eng = self._engine()
        tot, n = np.zeros(2), 0
        for i in range(0, len(x), batch_size):
            xb, yb = x[i:i + batch_size], y[i:i + batch_size]
            la = eng.evaluate_batch(self._to_dev(xb), self._to_dev(yb)).cpu().numpy()
            tot += la * len(xb)
            n += len(xb)
        return (tot / n).tolist()

    def fit(self, x, y, batch_size=32, epochs=1, verbose=1, callbacks=None, shuffle=True, distributed=None,
            **kw):
        """keras Model.fit.  The permutation is drawn from numpy's global RNG each epoch
        (as Keras does).  Distributed, ``batch_size`` is PER RANK, as for the generators
        (ImageDataGenerator.flow / flow_from_directory): every rank walks rank 0's
        permutation in global batches of batch_size * world frames and trains on its
        contiguous share; a global batch with fewer frames than ranks is dropped."""
        if distributed or (distributed is None and self._dp is None and _dist_world() > 1):
            self.distribute()
        r, w = self.world

        def perm():
            idx = np.random.permutation(len(x)) if shuffle else np.arange(len(x))
            if w > 1:
                import torch.distributed as tdist
                box = [idx]
                tdist.broadcast_object_list(box, src=0, group=self._dp_args[1])
                idx = box[0]
            return idx

        gb = batch_size * w

        class _Gen:
            last_global_batch = None

            def __iter__(self):
                return self

            def __next__(self):
                return next(it)

        g = _Gen()

        def batches():
            while True:
                idx = perm()
                for i in range(0, len(x), gb):
                    blk = idx[i:i + gb]
                    if len(blk) < w:
                        continue
                    g.last_global_batch = len(blk)
                    j = np.array_split(blk, w)[r]
                    yield x[j], y[j]
        it = batches()
        steps = sum(1 for i in range(0, len(x), gb) if len(x) - i >= w)
        return self.fit_generator(g, steps_per_epoch=steps, epochs=epochs, verbose=verbose,
                                  callbacks=callbacks)

    def fit_generator(self, generator, steps_per_epoch=None, epochs=1, verbose=1, callbacks=None,
                      validation_data=None, validation_steps=None, initial_epoch=0, distributed=None,
                      **kwargs):
        """keras Model.fit_generator (main.py:126-132): generator yields (x, y) batches.

        Epoch loss/acc are means over samples (per-step values weighted by batch size,
        as Keras does).  A generator exposing ``last_global_batch`` (the rank-sharded
        ImageDataGenerator iterators, or a ``zip`` of two of them) gets global-batch-mean
        gradients under data parallelism (see train_on_batch).  ``distributed=True`` (or None with an initialised process group
        of more than one rank) trains data-parallel: each rank consumes its own
        generator, logs are averaged over all ranks' samples, callbacks run on rank 0
        only and a ``stop_training`` raised there stops every rank."""
        self._check_compiled()
        if distributed or (distributed is None and self._dp is None and _dist_world() > 1):
            self.distribute()
        rank, world = self.world
        from .callbacks import CallbackList
        cbs = CallbackList((callbacks or []) if rank == 0 else [], self)
        hist = History()
        self.stop_training = False
        cbs.call("on_train_begin", {})
        for epoch in range(initial_epoch, epochs):
            cbs.call("on_epoch_begin", epoch, {})
            t0 = time.time()
            pending = []
            for step in range(steps_per_epoch):
                xb, yb = next(generator)
                cbs.call("on_batch_begin", step, {"batch": step, "size": len(xb)})
                la = self.train_on_batch(xb, yb, sync=False, global_batch=_global_batch(generator))
                pending.append((la, len(xb)))
                cbs.call("on_batch_end", step, {"batch": step, "size": len(xb)})
            tot = np.zeros(3)
            for la, nb in pending:
                tot[:2] += la.cpu().numpy() * nb
                tot[2] += nb
            tot = self._allreduce_sum(tot)
            logs = {"loss": tot[0] / tot[2], "acc": tot[1] / tot[2]}
            if validation_data is not None:
                vt = np.zeros(3)
                vsteps = validation_steps or 1
                for _ in range(vsteps):
                    xv, yv = next(validation_data) if hasattr(validation_data, "__next__") else validation_data
                    vt[:2] += np.asarray(self.evaluate(xv, yv, batch_size=len(xv))) * len(xv)
                    vt[2] += len(xv)
                vt = self._allreduce_sum(vt)
                logs["val_loss"], logs["val_acc"] = vt[0] / vt[2], vt[1] / vt[2]
            if verbose and rank == 0:
                msg = " - ".join(f"{k}: {v:.4f}" for k, v in logs.items())
                print(f"Epoch {epoch + 1}/{epochs} - {time.time() - t0:.1f}s - {msg}", file=sys.stderr)
            hist.epoch.append(epoch)
            for k, v in logs.items():
                hist.history.setdefault(k, []).append(v)
            cbs.call("on_epoch_end", epoch, logs)
            if world > 1:
                self.stop_training = bool(self._allreduce_sum([float(self.stop_training)])[0])
            if self.stop_training:
                break
        cbs.call("on_train_end", {})
        return hist

    # ---- summary -------------------------------------------------------------------
    def summary(self, line_length=98, print_fn=print):
        """Keras-style table; totals reproduce /root/reference/layers.txt:140-142."""
        pos = [32, 53, 65, 98]
        head = ["Layer (type)", "Output Shape", "Param #", "Connected to"]

        def row(fields):
            line = ""
            for i, f in enumerate(fields):
                if i > 0:
                    line = line[:-1] + " "
                line += str(f)
                line = line[:pos[i]]
                line += " " * (pos[i] - len(line))
            print_fn(line.rstrip())

        print_fn("_" * line_length)
        row(head)
        print_fn("=" * line_length)
        for k, l in enumerate(self.layers):
            shp = "(None, " + ", ".join(str(d) for d in l.output.shape) + ")"
            conns = [f"{t.layer.name}[0][0]" for t in l.inbound] or [""]
            row([f"{l.name} ({l.type_name})", shp, l.count_params(), conns[0]])
            for c in conns[1:]:
                row(["", "", "", c])
            print_fn(("=" if k == len(self.layers) - 1 else "_") * line_length)
        total = self.count_params()
        nontrain = sum(int(np.prod(s)) for l in self.layers for _, s, tr in l.weight_shapes() if not tr)
        print_fn(f"Total params: {total:,}")
        print_fn(f"Trainable params: {total - nontrain:,}")
        print_fn(f"Non-trainable params: {nontrain:,}")
        print_fn("_" * line_length)

    # ---- persistence -----------------------------------------------------------------
    def get_config(self):
        nodes = []
        for l in self.layers:
            nodes.append({"class": l.type_name, "config": l.get_config(),
                          "inbound": [t.layer.name for t in l.inbound]})
        return {"name": self.name, "layers": nodes, "input": self.inputs[0].layer.name,
                "output": self.outputs[0].layer.name}

    def named_accumulators(self):
        """RMSprop accumulators per trainable weight (internal layout), or None before
        the first step / without an optimizer state."""
        pending = getattr(self, "_pending_accum", None)
        if self.engine is None:
            if pending is not None and isinstance(pending[0], str):
                return {k: v.copy() for k, v in pending[1].items()}
            return None
        acc = self.engine.accum.cpu().numpy()
        return {k: acc[off:off + int(np.prod(shp))].reshape(shp).copy()
                for k, (off, shp) in self.engine.pslices.items()}

    @staticmethod
    def _is_h5_path(path):
        return str(path).lower().endswith((".h5", ".hdf5", ".keras", ".hdf"))

    def save(self, path, include_optimizer=True):
        """``*.h5`` / ``*.hdf5``: the Keras 2.2 HDF5 layout the reference's ModelCheckpoint
        writes (main.py:124; keras_h5.py).  Any other path: architecture + weights
        (+ RMSprop accumulators) in one .npz."""
        if self._is_h5_path(path):
            from . import keras_h5
            keras_h5.save_model_hdf5(self, path, include_optimizer=include_optimizer)
            return
        arrays = {"__config__": np.frombuffer(json.dumps(self.get_config()).encode(), np.uint8)}
        for k, v in self.named_weights().items():
            arrays["w/" + k] = v
        if include_optimizer and self.engine is not None:
            arrays["opt/accum"] = self.engine.accum.cpu().numpy()
            arrays["opt/step"] = np.array([self.engine.step])
            arrays["opt/dtype"] = np.frombuffer(self.dtype.encode(), np.uint8)
        if self.optimizer is not None:
            arrays["opt/hyper"] = np.array([self.optimizer.lr, self.optimizer.rho, self.optimizer.epsilon])
        tmp = path + ".tmp.npz"
        np.savez(tmp, **arrays)
        os.replace(tmp, path)

    def save_weights(self, path):
        if self._is_h5_path(path):
            from . import keras_h5
            keras_h5.save_model_hdf5(self, path, weights_only=True)
            return
        self.save(path, include_optimizer=False)

    def load_weights(self, path, by_name=False):
        """keras Model.load_weights: HDF5 weights are matched topologically (file layer k
        -> k-th model layer with weights), or by layer name with ``by_name=True``."""
        from . import hdf5
        if hdf5.is_hdf5(path):
            from . import keras_h5
            keras_h5.load_weights_hdf5(self, path, by_name=by_name)
            return
        with np.load(path, allow_pickle=False) as z:
            self.set_named_weights({k[2:]: z[k] for k in z.files if k.startswith("w/")})


def _global_batch(gen):
    """Frames of the global batch just drawn over all ranks: the generator's own
    ``last_global_batch`` (rank-sharded iterators, Model.fit); for the reference's
    builtin ``zip(input, target)`` (main.py:99), the members' values when every member
    is a rank-sharded datagen Iterator and they agree; otherwise None (the mean of the
    ranks' batch means).  A wrapper that prefetches or merges draws is not a zip of
    iterators, so it never borrows a count that belongs to another batch."""
    v = getattr(gen, "last_global_batch", None)
    if v is not None:
        return v
    if type(gen) is zip:
        from .datagen import Iterator
        members = gen.__reduce__()[1]  # zip pickles as (zip, (iterator, ...))
        if members and all(isinstance(m, Iterator) for m in members):
            vals = {m.last_global_batch for m in members}
            if len(vals) == 1:
                return vals.pop()
    return None


def _dist_world():
    try:
        import torch.distributed as tdist
        return tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1
    except ImportError:  # pragma: no cover
        return 1


def load_model(path, compile=True):
    """keras.models.load_model (predict.py:24): a Keras 2.2 HDF5 model file (as the
    reference's ModelCheckpoint writes it) or an .npz written by Model.save."""
    from . import hdf5
    if hdf5.is_hdf5(path):
        from . import keras_h5
        return keras_h5.load_model_hdf5(path, compile=compile)
    from . import layers as Lm
    with np.load(path, allow_pickle=False) as z:
        cfg = json.loads(bytes(z["__config__"]).decode())
        built = {}
        for node in cfg["layers"]:
            cls = Lm.LAYER_CLASSES[node["class"]]
            c = dict(node["config"])
            if cls is InputLayer:
                built[c["name"]] = Lm.InputLayer(c["shape"], name=c["name"]).output
                continue
            layer = cls(**c)
            ins = [built[n] for n in node["inbound"]]
            built[c["name"]] = layer(ins if len(ins) > 1 else ins[0])
        m = Model(inputs=built[cfg["input"]], outputs=built[cfg["output"]], name=cfg["name"])
        m.set_named_weights({k[2:]: z[k] for k in z.files if k.startswith("w/")})
        if compile and "opt/hyper" in z.files:
            lr, rho, eps = z["opt/hyper"].tolist()
            m.compile(RMSprop(lr=lr, rho=rho, epsilon=eps), "mse", ["accuracy"])
        if "opt/dtype" in z.files:
            m.dtype = bytes(z["opt/dtype"]).decode()
        if "opt/accum" in z.files:
            m._pending_accum = (z["opt/accum"].copy(), int(z["opt/step"][0]))
    return m
