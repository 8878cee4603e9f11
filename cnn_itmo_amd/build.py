"""Build libcnnitmo.so (all HIP kernels + the C ABI) in-tree for gfx950.

    python -m cnn_itmo_amd.build [--force] [-j N]

Each csrc/*.hip is compiled separately with hipcc (cached by mtime against its
sources) and linked into cnn_itmo_amd/lib/libcnnitmo.so.  No CMake, no JIT
cache outside the repo: the .so travels with the tree to the GPU box.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libcnnitmo.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CNNITMO_ARCH", "gfx950")

CFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
    "-Wno-unused-variable", "-munsafe-fp-atomics", f"-I{os.path.join(ROOT, 'include')}",
]


def _deps():
    return glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "cnn_itmo.h")]


def _stale(obj, src, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _compile(src, obj):
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    deps = _deps()
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.basename(s)[:-4] + ".o")
        objs.append(o)
        if force or _stale(o, s, deps):
            todo.append((s, o))
    if todo:
        if verbose:
            print(f"[cnnitmo build] compiling {len(todo)} file(s) for {ARCH}", file=sys.stderr)
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(lambda so: _compile(*so), todo))
    if todo or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=4)
    a = ap.parse_args()
    print(build(a.force, a.j))
