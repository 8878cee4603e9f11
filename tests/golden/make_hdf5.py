"""Generate tests/golden/keras_tinynet.hdf5 with the REAL HDF5 C library (libhdf5
1.10 via tests/h5lib.py), in the layout Keras 2.2.4 ``Model.save`` writes through
h5py (earliest file format, fixed-length string attributes, contiguous
datasets, RMSprop optimizer_weights), plus the expected Keras-layout arrays in
keras_tinynet_expected.npz.  The fixture pins cnn_itmo_amd/hdf5.py's reader
against a file it did not write; run once here (needs libhdf5):

    python tests/golden/make_hdf5.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import h5lib  # noqa: E402
import cnn_itmo_amd as C  # noqa: E402


def main():
    assert h5lib.load() is not None, "libhdf5 not found"
    C.clear_session()
    m = C.TinyNet(seed=3)
    rng = np.random.default_rng(11)
    accum = [rng.uniform(0, 1e-3, size=w.shape).astype(np.float32) for w in m.get_weights()]
    path = os.path.join(HERE, "keras_tinynet.hdf5")
    h5lib.write_keras_model(path, m, optimizer=accum)
    ws = m.get_weights()
    np.savez(os.path.join(HERE, "keras_tinynet_expected.npz"),
             **{f"w{i}": w for i, w in enumerate(ws)}, **{f"a{i}": a for i, a in enumerate(accum)})
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
