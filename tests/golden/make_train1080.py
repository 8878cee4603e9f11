"""Fixture tests/golden/train1080.npz: ONE training step of the U-Net at the benchmarked frame
size (1080x1920, padded to 1088 rows), restated by the fp64 oracle, and the deviation from it of
numpy-fp32 (the noise floor an fp32 implementation is held to) and of the bf16-storage oracle
(fp64 arithmetic, every stored tensor rounded to bf16: the floor of the bf16 bench dtype).

    python tools/train1080_oracle.py --out /tmp/o64.npz --dtype float64
    python tools/train1080_oracle.py --out /tmp/o32.npz --dtype float32
    python tools/train1080_oracle.py --out /tmp/o16.npz --dtype bf16store
    python tests/golden/make_train1080.py /tmp/o64.npz /tmp/o32.npz /tmp/o16.npz

The inputs are tools/train1080_oracle.inputs() (the 12 reference SDR frames tiled into one
1080x1920 mosaic, sdr1080.npz's seeded weights, a seeded tone-curve target, dropout seed 5).
Stored per gradient tensor g (fp64 oracle): its L2 norm; all values when it has at most
4096 entries, else the values at 4096 fixed random indices (a rel-L2 estimate within a few
per cent); the rel-L2 of numpy-fp32's g (floor/) and of the bf16-storage g (floor16/).  Loss /
accuracy of every run; the moving statistics
after the step in full.  (~1 MB instead of the 89 MB of full fp64 gradients.)
"""
import os
import sys

import numpy as np

S = 4096


def main(f64, f32, f16):
    a, b, c = np.load(f64), np.load(f32), np.load(f16)
    d = {"loss64": a["loss"], "loss32": b["loss"], "loss16": c["loss"], "acc64": a["acc"], "acc32": b["acc"],
         "acc16": c["acc"], "samples": np.array(S)}
    rng = np.random.default_rng(1088)
    for k in sorted(a.files):
        if not (k.startswith("g/") or k.startswith("m/")):
            continue
        x, y, z = a[k].reshape(-1), b[k].reshape(-1), c[k].reshape(-1)
        nx = float(np.linalg.norm(x))
        d["norm/" + k] = np.array(nx)
        d["floor/" + k] = np.array(float(np.linalg.norm(x - y)) / max(nx, 1e-300))
        d["floor16/" + k] = np.array(float(np.linalg.norm(x - z)) / max(nx, 1e-300))
        if x.size <= S or k.startswith("m/"):
            d["val/" + k] = x
        else:
            idx = np.sort(rng.choice(x.size, S, replace=False)).astype(np.int64)
            d["idx/" + k] = idx
            d["val/" + k] = x[idx]
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "train1080.npz")
    np.savez_compressed(out, **d)
    print(out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
