"""Minimal keras.callbacks equivalents used by the reference's train loop
(main.py:69,121,123-124): CSVLogger, ModelCheckpoint, LambdaCallback."""
from __future__ import annotations

import csv
import os


class Callback:
    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_batch_begin(self, batch, logs=None): pass
    def on_batch_end(self, batch, logs=None): pass


class CallbackList:
    def __init__(self, cbs, model):
        self.cbs = list(cbs)
        for c in self.cbs:
            c.set_model(model)

    def call(self, name, *args):
        for c in self.cbs:
            getattr(c, name)(*args)


class LambdaCallback(Callback):
    def __init__(self, on_epoch_begin=None, on_epoch_end=None, on_batch_begin=None, on_batch_end=None,
                 on_train_begin=None, on_train_end=None):
        self._f = dict(on_epoch_begin=on_epoch_begin, on_epoch_end=on_epoch_end,
                       on_batch_begin=on_batch_begin, on_batch_end=on_batch_end,
                       on_train_begin=on_train_begin, on_train_end=on_train_end)
        for k, f in self._f.items():
            if f is not None:
                setattr(self, k, f)


class CSVLogger(Callback):
    """CSVLogger('log.csv', append=True, separator=';') -- main.py:121."""

    def __init__(self, filename, separator=",", append=False):
        self.filename, self.sep, self.append = filename, separator, append
        self.keys = None

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        if self.keys is None:
            self.keys = sorted(logs)
        new = not (self.append and os.path.exists(self.filename) and os.path.getsize(self.filename) > 0)
        mode = "a" if self.append else ("w" if epoch == 0 else "a")
        with open(self.filename, mode, newline="") as f:
            w = csv.writer(f, delimiter=self.sep)
            if new and (self.append or epoch == 0):
                w.writerow(["epoch"] + self.keys)
            w.writerow([epoch] + [logs.get(k, "") for k in self.keys])


class ModelCheckpoint(Callback):
    """ModelCheckpoint(filepath) -- main.py:123-124; filepath may use {epoch} and log keys."""

    def __init__(self, filepath, monitor="val_loss", verbose=0, save_best_only=False, mode="auto",
                 save_weights_only=False, period=1):
        self.filepath, self.verbose, self.weights_only, self.period = filepath, verbose, save_weights_only, period

    def on_epoch_end(self, epoch, logs=None):
        if (epoch + 1) % self.period:
            return
        path = self.filepath.format(epoch=epoch + 1, **(logs or {}))
        (self.model.save_weights if self.weights_only else self.model.save)(path)
        if self.verbose:
            print(f"Epoch {epoch + 1}: saving model to {path}")
