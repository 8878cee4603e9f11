"""ctypes binding to the real HDF5 C library (test infrastructure only).

The image carries libhdf5 1.10 (``/opt/conda/lib/libhdf5.so``; override with
CNNITMO_LIBHDF5) but no h5py.  The tests use it as the independent checker of
cnn_itmo_amd/hdf5.py: files written by the library are read by our reader, and
files written by our writer are read back by the library.  ``load()`` returns
None when the library is absent (the tests then skip)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

H5F_ACC_RDONLY, H5F_ACC_TRUNC = 0, 2
H5P_DEFAULT, H5S_ALL, H5S_SCALAR = 0, 0, 0
H5T_STR_NULLPAD = 1
H5T_VARIABLE = C.c_size_t(-1).value

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("CNNITMO_LIBHDF5", "/opt/conda/lib/libhdf5.so")
    try:
        lib = C.CDLL(path)
    except OSError:
        return None
    i64, u64p = C.c_int64, C.POINTER(C.c_uint64)
    sig = {
        "H5open": (C.c_int, []),
        "H5Fcreate": (i64, [C.c_char_p, C.c_uint, i64, i64]),
        "H5Fopen": (i64, [C.c_char_p, C.c_uint, i64]),
        "H5Fclose": (C.c_int, [i64]),
        "H5Gcreate2": (i64, [i64, C.c_char_p, i64, i64, i64]),
        "H5Gopen2": (i64, [i64, C.c_char_p, i64]),
        "H5Gclose": (C.c_int, [i64]),
        "H5Screate_simple": (i64, [C.c_int, u64p, u64p]),
        "H5Screate": (i64, [C.c_int]),
        "H5Sclose": (C.c_int, [i64]),
        "H5Sget_simple_extent_ndims": (C.c_int, [i64]),
        "H5Sget_simple_extent_dims": (C.c_int, [i64, u64p, u64p]),
        "H5Dcreate2": (i64, [i64, C.c_char_p, i64, i64, i64, i64, i64]),
        "H5Dopen2": (i64, [i64, C.c_char_p, i64]),
        "H5Dwrite": (C.c_int, [i64, i64, i64, i64, i64, C.c_void_p]),
        "H5Dread": (C.c_int, [i64, i64, i64, i64, i64, C.c_void_p]),
        "H5Dget_space": (i64, [i64]),
        "H5Dclose": (C.c_int, [i64]),
        "H5Acreate2": (i64, [i64, C.c_char_p, i64, i64, i64, i64]),
        "H5Aopen": (i64, [i64, C.c_char_p, i64]),
        "H5Awrite": (C.c_int, [i64, i64, C.c_void_p]),
        "H5Aread": (C.c_int, [i64, i64, C.c_void_p]),
        "H5Aget_type": (i64, [i64]),
        "H5Aget_space": (i64, [i64]),
        "H5Aclose": (C.c_int, [i64]),
        "H5Tcopy": (i64, [i64]),
        "H5Tset_size": (C.c_int, [i64, C.c_size_t]),
        "H5Tget_size": (C.c_size_t, [i64]),
        "H5Tset_strpad": (C.c_int, [i64, C.c_int]),
        "H5Tclose": (C.c_int, [i64]),
        "H5Pcreate": (i64, [i64]),
        "H5Pset_chunk": (C.c_int, [i64, C.c_int, u64p]),
        "H5Pset_deflate": (C.c_int, [i64, C.c_uint]),
        "H5Pset_shuffle": (C.c_int, [i64]),
        "H5Pset_libver_bounds": (C.c_int, [i64, C.c_int, C.c_int]),
        "H5Pclose": (C.c_int, [i64]),
    }
    for n, (res, args) in sig.items():
        f = getattr(lib, n)
        f.restype, f.argtypes = res, args
    if lib.H5open() < 0:
        return None
    _lib = lib
    return lib


def _g(name):
    return C.c_int64.in_dll(_lib, name).value


def _dims(shape):
    return (C.c_uint64 * max(len(shape), 1))(*shape)


def _ok(v, what):
    if v < 0:
        raise RuntimeError(f"libhdf5: {what} failed")
    return v


class LibFile:
    """Minimal writer/reader over the C API: groups by path, float datasets,
    fixed- or variable-length string attributes."""

    def __init__(self, path, mode="r", latest=False, chunked=False):
        self.lib = L = load()
        self.chunked = chunked
        if mode == "w":
            fapl = H5P_DEFAULT
            if latest:
                fapl = L.H5Pcreate(_g("H5P_CLS_FILE_ACCESS_ID_g"))
                L.H5Pset_libver_bounds(fapl, 2, 2)
            self.f = _ok(L.H5Fcreate(str(path).encode(), H5F_ACC_TRUNC, H5P_DEFAULT, fapl), "H5Fcreate")
            if fapl:
                L.H5Pclose(fapl)
        else:
            self.f = _ok(L.H5Fopen(str(path).encode(), H5F_ACC_RDONLY, H5P_DEFAULT), "H5Fopen")

    def close(self):
        self.lib.H5Fclose(self.f)

    def group(self, path):
        """Create every missing group along `path` (returns nothing; groups are closed)."""
        L = self.lib
        cur = ""
        for part in [p for p in path.split("/") if p]:
            cur += "/" + part
            g = L.H5Gopen2(self.f, cur.encode(), H5P_DEFAULT) if self._exists(cur) else \
                _ok(L.H5Gcreate2(self.f, cur.encode(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), "H5Gcreate2")
            L.H5Gclose(g)

    def _exists(self, path):
        # H5Lexists would need another binding; groups are created in order so track them
        self._made = getattr(self, "_made", set())
        if path in self._made:
            return True
        self._made.add(path)
        return False

    def dataset(self, path, arr):
        L = self.lib
        a = np.ascontiguousarray(arr, dtype=np.float32)
        parent = path.rsplit("/", 1)[0]
        if parent:
            self.group(parent)
        sp = L.H5Screate_simple(a.ndim, _dims(a.shape), None) if a.ndim else L.H5Screate(H5S_SCALAR)
        dcpl = H5P_DEFAULT
        if self.chunked and a.ndim:
            dcpl = L.H5Pcreate(_g("H5P_CLS_DATASET_CREATE_ID_g"))
            L.H5Pset_chunk(dcpl, a.ndim, _dims([max(1, (d + 1) // 2) for d in a.shape]))
            L.H5Pset_shuffle(dcpl)
            L.H5Pset_deflate(dcpl, 4)
        d = _ok(L.H5Dcreate2(self.f, path.encode(), _g("H5T_IEEE_F32LE_g"), sp, H5P_DEFAULT, dcpl, H5P_DEFAULT),
                "H5Dcreate2")
        _ok(L.H5Dwrite(d, _g("H5T_NATIVE_FLOAT_g"), H5S_ALL, H5S_ALL, H5P_DEFAULT, a.ctypes.data), "H5Dwrite")
        L.H5Dclose(d)
        L.H5Sclose(sp)
        if dcpl:
            L.H5Pclose(dcpl)

    def _obj(self, path):
        L = self.lib
        if path in ("", "/"):
            return L.H5Gopen2(self.f, b"/", H5P_DEFAULT), L.H5Gclose
        return _ok(L.H5Gopen2(self.f, path.encode(), H5P_DEFAULT), "H5Gopen2"), L.H5Gclose

    def attr(self, path, name, value, vlen=False):
        """value: bytes/str (scalar) or a list of bytes/str (1-D array)."""
        L = self.lib
        vals = value if isinstance(value, (list, tuple)) else [value]
        vals = [v.encode() if isinstance(v, str) else v for v in vals]
        t = L.H5Tcopy(_g("H5T_C_S1_g"))
        if vlen:
            L.H5Tset_size(t, H5T_VARIABLE)
            buf = (C.c_char_p * len(vals))(*vals)
        else:
            n = max(1, max(len(v) for v in vals))
            L.H5Tset_size(t, n)
            L.H5Tset_strpad(t, H5T_STR_NULLPAD)
            buf = C.create_string_buffer(b"".join(v.ljust(n, b"\0") for v in vals), n * len(vals))
        sp = L.H5Screate_simple(1, _dims([len(vals)]), None) if isinstance(value, (list, tuple)) \
            else L.H5Screate(H5S_SCALAR)
        o, close = self._obj(path)
        a = _ok(L.H5Acreate2(o, name.encode(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "H5Acreate2")
        _ok(L.H5Awrite(a, t, buf), "H5Awrite")
        L.H5Aclose(a)
        close(o)
        L.H5Sclose(sp)
        L.H5Tclose(t)

    def read_dataset(self, path):
        L = self.lib
        d = _ok(L.H5Dopen2(self.f, path.encode(), H5P_DEFAULT), "H5Dopen2")
        sp = L.H5Dget_space(d)
        nd = L.H5Sget_simple_extent_ndims(sp)
        dims = (C.c_uint64 * max(nd, 1))()
        L.H5Sget_simple_extent_dims(sp, dims, None)
        shape = tuple(dims[i] for i in range(nd))
        out = np.empty(shape, dtype=np.float32)
        _ok(L.H5Dread(d, _g("H5T_NATIVE_FLOAT_g"), H5S_ALL, H5S_ALL, H5P_DEFAULT, out.ctypes.data), "H5Dread")
        L.H5Sclose(sp)
        L.H5Dclose(d)
        return out

    def read_str_attr(self, path, name):
        """Fixed-length string attribute -> list of bytes (scalar: one element)."""
        L = self.lib
        o, close = self._obj(path)
        a = _ok(L.H5Aopen(o, name.encode(), H5P_DEFAULT), "H5Aopen")
        t = L.H5Aget_type(a)
        n = L.H5Tget_size(t)
        sp = L.H5Aget_space(a)
        nd = L.H5Sget_simple_extent_ndims(sp)
        dims = (C.c_uint64 * max(nd, 1))()
        L.H5Sget_simple_extent_dims(sp, dims, None)
        cnt = int(np.prod([dims[i] for i in range(nd)])) if nd else 1
        buf = C.create_string_buffer(n * cnt)
        _ok(L.H5Aread(a, t, buf), "H5Aread")
        L.H5Sclose(sp)
        L.H5Tclose(t)
        L.H5Aclose(a)
        close(o)
        raw = buf.raw
        return [raw[i * n:(i + 1) * n].rstrip(b"\0") for i in range(cnt)]


def write_keras_model(path, model, latest=False, chunked=False, vlen=False, optimizer=None):
    """Write `model` the way Keras 2.2.4 ``Model.save`` does through h5py (root attrs,
    /model_weights/<layer>/<layer>/<w>:0, weight_names, optimizer_weights), but with
    the HDF5 C library itself.  optimizer: list of Keras-layout accumulators or None."""
    import json
    from cnn_itmo_amd import keras_h5
    from cnn_itmo_amd.model import _to_keras
    f = LibFile(path, "w", latest=latest, chunked=chunked)
    f.attr("/", "keras_version", keras_h5.KERAS_VERSION, vlen=vlen)
    f.attr("/", "backend", "tensorflow", vlen=vlen)
    f.attr("/", "model_config", json.dumps(keras_h5.model_config(model)), vlen=vlen)
    f.group("/model_weights")
    f.attr("/model_weights", "layer_names", [l.name for l in model.layers], vlen=vlen)
    f.attr("/model_weights", "backend", "tensorflow", vlen=vlen)
    f.attr("/model_weights", "keras_version", keras_h5.KERAS_VERSION, vlen=vlen)
    named = model.named_weights()
    trainable = []
    for l in model.layers:
        g = "/model_weights/" + l.name
        f.group(g)
        names = [f"{l.name}/{w}:0" for w, _, _ in l.weight_shapes()]
        if names:
            f.attr(g, "weight_names", names, vlen=vlen)
        for (w, _, tr), nm in zip(l.weight_shapes(), names):
            f.dataset(g + "/" + nm, _to_keras(l, w, named[f"{l.name}/{w}"]))
            if tr:
                trainable.append(None)
    if optimizer is not None:
        f.attr("/", "training_config", json.dumps(keras_h5.training_config(model)), vlen=vlen)
        f.group("/optimizer_weights")
        names = ["training/RMSprop/Variable%s:0" % ("" if i == 0 else f"_{i}") for i in range(len(optimizer))]
        f.attr("/optimizer_weights", "weight_names", names, vlen=vlen)
        for nm, v in zip(names, optimizer):
            f.dataset("/optimizer_weights/" + nm, v)
    f.close()
