#!/usr/bin/env python
"""Benchmark: 1080p SDR->HDR U-Net training throughput on MI355X.

BASELINE.json metric: "1080p SDR->HDR frames/sec (fwd+bwd) at 1/2/4/8 MI355X;
MFMA % of peak".  Workload (BASELINE configs[2]/[3]): 1920x1080 frames padded to
1920x1088 (the U-Net needs multiples of 16), batch 32 per GPU, bf16
storage / fp32 accumulation, one step = forward + backward + RCCL gradient
all-reduce (N>1) + RMSprop, synthetic data (uniform /255 inputs and targets),
random-init weights of the reference architecture (model.py:204-281).

  python bench.py [--gpus N] [--steps K] [--warmup W]     (N>1: spawns N ranks itself)
  torchrun --nproc-per-node N bench.py --gpus N ...       (one rank per GPU, RCCL)

Prints ONE JSON line on rank 0.  `value` = frames/s over all ranks (weak
scaling: 32 frames per GPU per step), timed over K steps with no per-launch
instrumentation.  `roofline` is for the dominant kernel: a second pass of
min(K, 10) steps brackets every conv launch with HIP events on the stream it
runs on (its ms/step is reported beside).  `allreduce_exposed` (N>1) is the time
the compute stream waits for the RCCL buckets after backward.  `cpu_baseline`
times this repo's numpy oracle (oracle/unet_ref.py) on the host (rank 0, N=1).
`fp32_infer` is BASELINE configs[1] (1080p b8 fp32 inference) with its own
roofline and CPU baseline; `fp32_infer_b32` the north star's fp32 conv2d forward at
1080p batch 32; `k4_train` is configs[4] (3840x2160, bf16 training, 8 frames per
GPU = global 64 on 8 GPUs); `fp32_train` the reference's own precision (Keras fp32
training, 1080p, 8 frames per GPU).  Each secondary leg carries its own roofline.
"""
from __future__ import annotations

import argparse
import contextlib
import functools
import io
import json
import os
import re
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BF16_PEAK_TF = 2516.6   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md; spec ~2.5 PF dense)
F32_PEAK_TF = 157.3     # MI355X fp32 MFMA (= fp32 vector rate)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float32"])
    ap.add_argument("--mode", default="train", choices=["train", "infer"])
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-scale", type=int, default=2, help="CPU sample = 1 frame at H/s x W/s")
    ap.add_argument("--bucket-mb", type=float, default=16.0)
    ap.add_argument("--infer-batch", type=int, default=8,
                    help="fp32 inference leg (configs[1]) frames per GPU; 0 = skip")
    ap.add_argument("--k4-batch", type=int, default=8,
                    help="4K bf16 training leg (configs[4]: 3840x2160, global 64 on 8 GPUs) frames per GPU; 0 = skip")
    ap.add_argument("--k4-steps", type=int, default=10)
    ap.add_argument("--k4-warmup", type=int, default=3)
    ap.add_argument("--f32-train-batch", type=int, default=8,
                    help="fp32 1080p training leg (the reference's Keras precision) frames per GPU; 0 = skip")
    ap.add_argument("--f32-train-steps", type=int, default=10)
    ap.add_argument("--f32-train-warmup", type=int, default=3)
    ap.add_argument("--ns-batch", type=int, default=32,
                    help="north-star leg: fp32 1080p inference (conv2d forward) at this batch per GPU; 0 = skip")
    return ap.parse_args()


# ---------------------------------------------------------------- kernel timing
class KernelTimer:
    """Brackets every launch of the implicit-GEMM conv kernels with HIP events on
    the current (compute) stream and attributes algorithmic FLOPs to the kernel
    instantiation that runs (same tile choice as csrc/igemm_fwd.hip:pick_cfg)."""

    def __init__(self, ops, torch):
        self.ops, self.torch = ops, torch
        self.on = False
        self.rec = []  # (name, flops, ev0, ev1, tag, algorithmic bytes)
        self._nb = 0  # algorithmic HBM bytes of the next bracketed launch (conv3x3 fwd only)
        self._pool, self._next = [], 0
        self._wrap()

    @staticmethod
    def fwd_name(dt, n):
        """Kernel chosen by igemm_fwd.hip's dispatch for n GEMM columns (mirrors pick2)."""
        t = "bf16" if dt == 1 else "f32"
        if n == 32:
            return f"igemm_fwd_kernel<{t},256x32>"
        bn = 128 if n % 128 == 0 else 64 if n % 64 == 0 else 96 if n % 96 == 0 else 32
        return f"igemm_fwd2_kernel<{t},256x{bn}>"

    def _bracket(self, name, flops, tag, fn, *a, **k):
        nb, self._nb = self._nb, 0
        if not self.on:
            return fn(*a, **k)
        i = self._next
        if i == len(self._pool):  # events are created once and reused pass after pass
            self._pool.append((self.torch.cuda.Event(enable_timing=True), self.torch.cuda.Event(enable_timing=True)))
        e0, e1 = self._pool[i]
        self._next += 1
        e0.record()
        r = fn(*a, **k)
        e1.record()
        self.rec.append((name, flops, e0, e1, tag, nb))
        return r

    def reset(self):
        self.rec = []
        self._next = 0

    def _wrap(self):
        ops = self.ops
        query = functools.lru_cache(maxsize=None)(ops.query)  # kernel names: one ctypes query per shape
        o = {n: getattr(ops, n) for n in ("conv3x3_fwd", "conv3x3_fwd_pool", "conv3x3_fwd_head", "conv3x3_fwd_cat", "conv_wgrad_cat", "conv3x3_dgrad", "conv3x3_dgrad_bn", "conv3x3_dgrad_bn_pooled",
                                           "tconv_fwd", "tconv_dgrad", "tconv_dgrad_bn", "conv1tap_fwd", "conv_wgrad",
                                           "tconv_wgrad", "conv_c3_fwd", "conv_c3_wgrad")}

        def kname(dt, n, h, w, cin, cout, dgrad):
            return query("cnnitmo_conv3x3_kernel_name", dt, n, h, w, cin, cout, dgrad).decode()

        def conv3x3_fwd(dt, x, wt, bias, out, *a, **k):
            fl = 2.0 * x.p * out.c * 9 * x.c
            # single-pass bytes: the input view once, the output once, the weights once (also tconv_fwd)
            self._nb = (2 if dt == 1 else 4) * (x.p * x.c + x.p * out.c + 9 * x.c * out.c)
            return self._bracket(kname(dt, x.n, x.h, x.w, x.c, out.c, 0), fl, f"fwd {x.h}x{x.w} {x.c}->{out.c}", o["conv3x3_fwd"], dt, x, wt, bias,
                                 out, *a, **k)

        def conv3x3_fwd_pool(dt, x, wt, bias, out, *a, **k):
            fl = 2.0 * x.p * out.c * 9 * x.c
            # + the pooled value and window index it writes (the stand-alone pool pass it replaces)
            self._nb = (2 if dt == 1 else 4) * (x.p * x.c + x.p * out.c + 9 * x.c * out.c) + \
                ((2 if dt == 1 else 4) + 1) * x.p * out.c // 4
            nm = kname(dt, x.n, x.h, x.w, x.c, out.c, 0).replace(">", ",pool>")
            return self._bracket(nm, fl, f"fwd+pool {x.h}x{x.w} {x.c}->{out.c}", o["conv3x3_fwd_pool"], dt, x, wt,
                                 bias, out, *a, **k)

        def conv3x3_fwd_head(dt, x, wt, bias, cout, flags, aff, h_valid, head_w, head_b, yhat):
            # the conv's FLOPs + the 1x1 cout->3 head; bytes: input, weights and the fp32 yhat
            fl = 2.0 * x.p * cout * 9 * x.c + 2.0 * x.n * h_valid * x.w * 3 * cout
            self._nb = (2 if dt == 1 else 4) * (x.p * x.c + 9 * x.c * cout) + 4 * 3 * x.n * h_valid * x.w
            nm = re.sub(r",1([,>])", r",3\1", kname(dt, x.n, x.h, x.w, x.c, cout, 0), count=1)
            return self._bracket(nm, fl, f"fwd+head {x.h}x{x.w} {x.c}->{cout}->3", o["conv3x3_fwd_head"], dt, x, wt,
                                 bias, cout, flags, aff, h_valid, head_w, head_b, yhat)

        def conv3x3_fwd_cat(dt, x1, x2, wt, bias, out, *a, **k):
            cin = x1.c + x2.c
            fl = 2.0 * x1.p * out.c * 9 * cin
            self._nb = 2 * (x1.p * cin + x1.p * out.c + 9 * cin * out.c)
            return self._bracket(kname(dt, x1.n, x1.h, x1.w, cin, out.c, 0), fl,
                                 f"fwd {x1.h}x{x1.w} {x1.c}+{x2.c}->{out.c}", o["conv3x3_fwd_cat"], dt, x1, x2, wt, bias,
                                 out, *a, **k)

        def conv_wgrad_cat(dt, x1, x2, dz, cout, dw, *a, **k):
            cin = x1.c + x2.c
            fl = 2.0 * x1.p * cout * 9 * cin
            name = query("cnnitmo_wgrad_cat_kernel_name", x1.n, x1.h, x1.w, x1.c, cin, cout).decode() + " + slab_reduce"
            return self._bracket(name, fl, f"wgrad {x1.h}x{x1.w} {x1.c}+{x2.c}->{cout}", o["conv_wgrad_cat"], dt, x1, x2,
                                 dz, cout, dw, *a, **k)

        def conv3x3_dgrad(dt, dz, n, h, w, cout, wflip, cin, dx):
            fl = 2.0 * n * h * w * cin * 9 * cout
            return self._bracket(kname(dt, n, h, w, cin, cout, 1), fl, f"dgrad {h}x{w} {cout}->{cin}", o["conv3x3_dgrad"], dt, dz, n, h, w, cout,
                                 wflip, cin, dx)

        def conv3x3_dgrad_bn(dt, dz, n, h, w, cout, wflip, cin, dx, c0, c1, *a, **k):
            fl = 2.0 * n * h * w * cin * 9 * cout
            name = query("cnnitmo_conv3x3_dgrad_bn_kernel_name", dt, n, h, w, cout, cin, c0, c1).decode()
            return self._bracket(name, fl, f"dgrad_bn {h}x{w} {cout}->{cin}[{c0}:{c1}]", o["conv3x3_dgrad_bn"], dt, dz, n, h, w, cout, wflip, cin, dx, c0, c1,
                                 *a, **k)

        def conv3x3_dgrad_bn_pooled(dt, dz, n, h, w, cout, wflip, cin, *a, **k):
            fl = 2.0 * n * h * w * cin * 9 * cout
            name = query("cnnitmo_conv3x3_dgrad_bn_pooled_kernel_name", dt, n, h, w, cout, cin).decode()
            return self._bracket(name, fl, f"dgrad_bn+route {h}x{w} {cout}->{cin}", o["conv3x3_dgrad_bn_pooled"], dt, dz,
                                 n, h, w, cout, wflip, cin, *a, **k)

        def tconv_dgrad_bn(dt, dout, n, h, w, cout, kT, cin, *a, **k):
            fl = 2.0 * n * h * w * cin * 4 * cout
            name = query("cnnitmo_tconv2x2_dgrad_bn_kernel_name", dt, n, h, w, cout, cin).decode()
            return self._bracket(name, fl, f"t.dgrad_bn {h}x{w} {cout}->{cin}", o["tconv_dgrad_bn"], dt, dout, n, h, w, cout, kT, cin, *a, **k)

        def tname(dt, n, h, w, cin, cout, dgrad):
            return query("cnnitmo_tconv2x2_kernel_name", dt, n, h, w, cin, cout, dgrad).decode()

        def tconv_fwd(dt, x, k_, bias, out, *a, **k):
            fl = 2.0 * x.p * 4 * out.c * x.c
            self._nb = (2 if dt == 1 else 4) * (x.p * x.c + 4 * x.p * out.c + 4 * x.c * out.c)
            return self._bracket(tname(dt, x.n, x.h, x.w, x.c, out.c, 0), fl, f"t.fwd {x.h}x{x.w} {x.c}->{out.c}", o["tconv_fwd"], dt, x, k_, bias, out,
                                 *a, **k)

        def tconv_dgrad(dt, dout, n, h, w, cout, kT, cin, dx):
            fl = 2.0 * n * h * w * cin * 4 * cout
            return self._bracket(tname(dt, n, h, w, cin, cout, 1), fl, f"t.dgrad {h}x{w} {cout}->{cin}", o["tconv_dgrad"], dt, dout, n, h, w, cout,
                                 kT, cin, dx)

        def conv1tap_fwd(dt, cols, kk, m, wt, bias, out, *a, **k):
            fl = 2.0 * m * out.c * 27  # algorithmic K = 3x3x3 (the packed 32 has 5 zero columns)
            return self._bracket(self.fwd_name(dt, out.c), fl, "c3in fwd", o["conv1tap_fwd"], dt, cols, kk, m, wt, bias, out, *a, **k)

        def conv_c3_fwd(dt, x, n, hv, h, w, *a, **k):
            fl = 2.0 * n * h * w * 32 * 27
            return self._bracket("conv_c3_fwd_kernel" + ("<f32>" if dt == 0 else ""), fl, "c3 fwd", o["conv_c3_fwd"],
                                 dt, x, n, hv, h, w, *a, **k)

        def conv_c3_wgrad(dt, x, n, hv, h, w, *a, **k):
            fl = 2.0 * n * h * w * 32 * 27
            kn = "conv_c3_wgrad_f32_kernel + fold" if dt == 0 else "conv_c3_wgrad_kernel + fold"
            return self._bracket(kn, fl, "c3 wgrad", o["conv_c3_wgrad"], dt, x, n, hv, h, w, *a, **k)

        def wname(dt, ntaps, n, h, w, cin, cout):
            k = query("cnnitmo_wgrad_kernel_name", dt, ntaps, n, h, w, cin, cout).decode()
            return k + " + slab_reduce"

        def conv_wgrad(dt, ntaps, x, dz, cout, dw, *a, **k):
            fl = 2.0 * x.p * cout * (27 if ntaps == 1 else 9 * x.c)
            return self._bracket(wname(dt, ntaps, x.n, x.h, x.w, x.c, cout), fl, f"wgrad {x.h}x{x.w} {x.c}->{cout}", o["conv_wgrad"],
                                 dt, ntaps, x, dz, cout, dw, *a, **k)

        def tconv_wgrad(dt, x, dout, cout, dk, *a, **k):
            fl = 2.0 * x.p * 4 * cout * x.c
            return self._bracket(wname(dt, 4, x.n, x.h, x.w, x.c, cout), fl, f"t.wgrad {x.h}x{x.w} {x.c}->{cout}", o["tconv_wgrad"],
                                 dt, x, dout, cout, dk, *a, **k)

        for n, f in (("conv3x3_fwd", conv3x3_fwd), ("conv3x3_fwd_pool", conv3x3_fwd_pool),
                     ("conv3x3_fwd_head", conv3x3_fwd_head),
                     ("conv3x3_fwd_cat", conv3x3_fwd_cat), ("conv_wgrad_cat", conv_wgrad_cat),
                     ("conv3x3_dgrad", conv3x3_dgrad),
                     ("conv3x3_dgrad_bn", conv3x3_dgrad_bn), ("conv3x3_dgrad_bn_pooled", conv3x3_dgrad_bn_pooled),
                     ("tconv_fwd", tconv_fwd),
                     ("tconv_dgrad", tconv_dgrad), ("tconv_dgrad_bn", tconv_dgrad_bn), ("conv1tap_fwd", conv1tap_fwd), ("conv_wgrad", conv_wgrad),
                     ("tconv_wgrad", tconv_wgrad), ("conv_c3_fwd", conv_c3_fwd), ("conv_c3_wgrad", conv_c3_wgrad)):
            setattr(ops, n, f)

    def detail(self):
        """(name, launch tag) -> [launches, flops, ms]: per-layer view of the same events."""
        agg = {}
        for name, fl, e0, e1, tag, _ in self.rec:
            a = agg.setdefault((name, tag), [0, 0.0, 0.0])
            a[0] += 1
            a[1] += fl
            a[2] += e0.elapsed_time(e1)
        return agg

    def summary(self):
        agg = {}
        for name, fl, e0, e1, _, nb in self.rec:
            ms = e0.elapsed_time(e1)
            a = agg.setdefault(name, [0, 0.0, 0.0, 0.0, 0])
            a[0] += 1
            a[1] += fl
            a[2] += ms
            a[3] += nb
            a[4] += 1 if nb else 0
        return agg


# ---------------------------------------------------------------- CPU baseline
def _host_info():
    """(affinity cores, BLAS threads, CPU model) of this process's host."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    try:
        from threadpoolctl import threadpool_info
        blas = max([d.get("num_threads", 1) for d in threadpool_info()
                    if d.get("internal_api") in ("openblas", "mkl")] or [1])
    except Exception:  # pragma: no cover
        blas = int(os.environ.get("OMP_NUM_THREADS", "1"))
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:  # pragma: no cover
        pass
    return cores, blas, model


def cpu_baseline(args, P_init, H, W, train=True):
    """Time the numpy oracle (fp32, OpenBLAS sgemm, the box's CPU share) on ONE frame at
    (H/s, W/s): a training step (fwd+bwd) or an inference forward, repeated to >= 10 s; report
    1080p-frame-equivalents per second (FLOPs scale with pixel count)."""
    from oracle import unet_ref as R
    s = args.cpu_scale
    h, w = H // s, W // s
    h, w = h - h % 16, w - w % 16
    rng = np.random.default_rng(0)
    x = (rng.integers(0, 256, size=(1, h, w, 3)) / 255.0).astype(np.float32)
    t = (rng.integers(0, 256, size=(1, h, w, 3)) / 255.0).astype(np.float32)
    net = R.UNetRef(P_init, np.float32)
    cores, blas, model = _host_info()
    # the oracle runs its convs' row bands on R._POOL threads, each in BLAS: split the CPU share
    # between them so that the threads in use (band threads x BLAS threads) never exceed it
    pool0 = R._POOL
    R._POOL = bands = max(1, min(pool0, blas))
    per = max(1, blas // bands)
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=per, user_api="blas"):
        k, t0 = 0, time.perf_counter()
        while True:  # repeated to at least 10 s of CPU work
            net.forward(x, training=train, seed=0)
            if train:
                net.backward(t)
            k += 1
            if time.perf_counter() - t0 >= 10.0:
                break
        dt = (time.perf_counter() - t0) / k
    R._POOL = pool0
    frac = (h * w) / float(H * W)
    what = "train step (fwd+bwd)" if train else "inference forward (BN moving stats)"
    return {"value": frac / dt, "unit": "1080p frames/s (%s, fp32)" % ("fwd+bwd" if train else "fwd"),
            "cores": bands * per, "kind": "port",
            "sample": f"oracle/unet_ref.py numpy fp32 {what} on 1 frame {w}x{h} "
                      f"({frac:.4f} of a 1920x{H} frame, scaled by pixel count), {k} x {dt:.2f} s",
            "seconds": dt, "padded_h": H, "affinity_cores": cores, "blas_threads": per, "band_threads": bands,
            "cpu_model": model, "threads_note": THREADS_NOTE}


# `cores` is the thread count actually used.  The GPU box allots 16 host CPUs per GPU (the
# harness exports OMP_NUM_THREADS=16 and asks for pools of at most 16); sched_getaffinity
# there lists every core of the host (256), which are not ours.
THREADS_NOTE = ("cores = the box's CPU share per GPU (OMP_NUM_THREADS, 16 on the MI355X box) = the oracle's "
                "row-band threads x BLAS threads per band; affinity_cores counts the whole host")


def cpu_config1():
    """BASELINE configs[0]: the 64x64 3-conv net (conv3x3 3->32 + ReLU, conv3x3 32->32 + ReLU,
    conv1x1 32->3 + sigmoid), batch 1, fwd+bwd on the CPU oracle, repeated for ~2 s."""
    from oracle import unet_ref as R
    rng = np.random.default_rng(0)
    P = R.init_tiny_params(0, np.float32)
    x = (rng.integers(0, 256, size=(1, 64, 64, 3)) / 255.0).astype(np.float32)
    t = (rng.integers(0, 256, size=(1, 64, 64, 3)) / 255.0).astype(np.float32)
    net = R.TinyNetRef(P, np.float32)
    net.forward(x)
    net.backward(t)
    k, t0 = 0, time.perf_counter()
    while True:
        net.forward(x)
        net.backward(t)
        k += 1
        dt = time.perf_counter() - t0
        if dt > 2.0:
            break
    cores, blas, model = _host_info()
    return {"value": k / dt, "unit": "steps/s (64x64 patch, batch 1, fwd+bwd, fp32)", "cores": blas, "kind": "port",
            "sample": f"oracle/unet_ref.py TinyNetRef, {k} steps in {dt:.2f} s", "ms_per_step": 1e3 * dt / k,
            "gflop_per_step": round(3 * 2 * 64 * 64 * (27 * 32 + 288 * 32 + 32 * 3) / 1e9, 4)}


# ---------------------------------------------------------------- launcher
def _spawn_ranks(args):
    """`python bench.py --gpus N` without a torchrun environment: start N rank
    processes (fresh children, before this process touches the GPU) under
    torch.distributed.run on 127.0.0.1, relay rank 0's JSON line, exit with their
    status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd[1:6])} ...", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


# ---------------------------------------------------------------- legs
def _lib_sha():
    import hashlib
    from cnn_itmo_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _traffic(name, shape):
    """HBM bytes per launch of kernel `name` from profiles/pmc_traffic.json (rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.sh) -> (bytes or None, provenance).
    Reported only when that profile was taken of THIS library build at THIS shape."""
    pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc):
        return None, "no profiles/pmc_traffic.json"
    try:
        tab = json.load(open(pmc))
    except Exception as e:  # pragma: no cover
        return None, f"unreadable pmc_traffic.json: {e!r}"
    meta = tab.get("_meta", {})
    src = {"file": "profiles/pmc_traffic.json", "profile_lib_sha256": meta.get("lib_sha256"),
           "profile_shapes": meta.get("shapes")}
    ent = tab.get("per_shape", {}).get(shape, {}).get(name.split(" + ")[0])
    if ent is None and shape in (meta.get("shapes") or []):
        return None, dict(src, why_null="kernel not in the profile")
    if meta.get("lib_sha256") != _lib_sha():
        return None, dict(src, why_null="profile taken of another library build")
    if shape not in (meta.get("shapes") or []):
        return None, dict(src, why_null=f"profile shapes do not include {shape}")
    return ent.get("bytes_per_launch"), src


def _roofline(agg, steps, elapsed, peak, shape=None):
    dom = max(agg.items(), key=lambda kv: kv[1][2])
    name, (cnt, fl, ms, nbytes, nbcnt) = dom
    if nbcnt != cnt:  # bytes are accounted for the conv3x3 / tconv forwards only
        nbytes = 0
    achieved = fl / (ms * 1e-3) / 1e12
    step_flops = sum(v[1] for v in agg.values()) / steps
    traffic, tsrc = _traffic(name, shape)
    return {"bound": "mfma", "kernel": name, "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": tsrc,
            "launches": cnt, "avg_launch_ms": round(ms / cnt, 4),
            "algorithmic_flop_per_launch": fl / cnt,
            # single-pass HBM bytes (input, output, weights once) per launch, and the
            # measured traffic over it (re-read factor)
            "algorithmic_bytes_per_launch": nbytes / cnt if nbytes else None,
            "traffic_over_algorithmic": round(traffic / (nbytes / cnt), 3) if traffic and nbytes else None,
            "step_conv_tflops": round(step_flops / (elapsed / steps) / 1e12, 2),
            "step_mfma_frac": round(step_flops / (elapsed / steps) / 1e12 / peak, 4)}, step_flops


def _print_agg(agg, tag):
    for k, (c, f, m, _, _) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        print(f"[bench:{tag}] {k:55s} launches={c:5d} time={m:9.1f} ms  {f / (m * 1e-3) / 1e12:7.1f} TFLOP/s",
              file=sys.stderr)


def _print_detail(det, steps, tag):
    """Per launch site (kernel, layer shape): ms per step and TFLOP/s."""
    for (k, t), (c, f, m) in sorted(det.items(), key=lambda kv: -kv[1][2]):
        print(f"[bench:{tag}:site] {m / steps:7.3f} ms/step {f / (m * 1e-3) / 1e12:7.1f} TF/s  {k:42s} {t}",
              file=sys.stderr)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_spawn_ranks(args))
    import torch
    from cnn_itmo_amd import dist as D
    rank, world, local = D.init_from_env()
    if world != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a dp{world} "
                         f"number as dp{args.gpus}")
    torch.cuda.set_device(local)
    import cnn_itmo_amd as C
    from cnn_itmo_amd import ops

    H = -(-args.height // 16) * 16
    W = -(-args.width // 16) * 16
    with contextlib.redirect_stdout(io.StringIO()):
        model = C.U_net(input_size=(args.height, args.width, 3), pad=True, dtype=args.dtype, seed=0,
                        verbose=False)
    P_init = model.named_weights() if rank == 0 else None
    eng = model._engine()
    dp = None
    if world > 1:
        model.distribute(bucket_mb=args.bucket_mb)  # the public DP path (Model.fit_generator uses it)
        dp = model._dp
        pg_world = torch.distributed.get_world_size()
        if rank == 0:
            print(f"[bench] process group: backend={torch.distributed.get_backend()} world_size={pg_world}, "
                  f"{len(dp.buckets)} gradient buckets", file=sys.stderr)
    timer = KernelTimer(ops, torch)

    g = torch.Generator(device="cuda")
    g.manual_seed(1234 + 7919 * rank)
    B = args.batch
    x = torch.randint(0, 256, (B, args.height, args.width, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
    t = torch.randint(0, 256, (B, args.height, args.width, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
    opt = model.optimizer

    def step(i):
        if args.mode == "infer":
            yhat = torch.empty(B, args.height, args.width, 3, device="cuda", dtype=torch.float32)
            eng.predict_into(x, yhat)  # Model.predict's path (fused head included)
            return None
        kw = dict(seed=i * world + rank, lr=opt.lr, rho=opt.rho, eps=opt.epsilon)
        if dp is not None:
            kw.update(sync=dp.finish, grad_scale=dp.grad_scale)
        return eng.train_step(x, t, **kw)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    def timed(n, first):
        barrier()
        t0 = time.perf_counter()
        out = [step(first + i) for i in range(n)]
        barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        return el.item(), out

    for i in range(args.warmup):
        step(i)
    # pass 1: throughput (no per-launch instrumentation inside the timed region)
    elapsed, losses = timed(args.steps, args.warmup)
    frames = B * world * args.steps
    fps = frames / elapsed
    # pass 2: the same steps with every conv launch bracketed by HIP events (roofline),
    # and the all-reduce wait left exposed on the compute stream after overlap
    timer.reset()
    timer.on = True
    if dp is not None:
        dp.timing = True
    k2 = max(1, min(args.steps, 10))
    elapsed2, _ = timed(k2, args.warmup + args.steps)
    timer.on = False
    exposed = None
    if dp is not None:
        dp.timing = False
        tot, n = dp.exposed_ms()
        exposed = {"ms_per_step": round(tot / max(n, 1), 3), "steps": n, "buckets": len(dp.buckets),
                   "bucket_mb": args.bucket_mb, "backend": torch.distributed.get_backend(),
                   "world_size": torch.distributed.get_world_size()}

    agg = timer.summary()
    peak = BF16_PEAK_TF if args.dtype == "bfloat16" else F32_PEAK_TF
    roof, step_flops = _roofline(agg, k2, elapsed2, peak, _shape(args.mode, args.height, args.width, B, args.dtype))
    roof["timed_pass_ms_per_step"] = round(elapsed2 / k2 * 1e3, 2)
    if rank == 0:
        _print_agg(agg, args.mode)
        _print_detail(timer.detail(), k2, args.mode)
        if losses and losses[-1] is not None:
            print(f"[bench] last loss/acc: {losses[-1].cpu().numpy().tolist()}", file=sys.stderr)
        print(f"[bench] peak mem {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB, "
              f"step {elapsed / args.steps * 1e3:.1f} ms (instrumented pass {elapsed2 / k2 * 1e3:.1f} ms)"
              + (f", exposed all-reduce {exposed['ms_per_step']} ms/step" if exposed else ""), file=sys.stderr)

    replicas = None
    if world > 1:  # DP correctness: every rank must hold the same parameters and moving stats
        import hashlib
        torch.cuda.synchronize()
        dig = hashlib.sha256(eng.params.cpu().numpy().tobytes() + eng.bufs.cpu().numpy().tobytes()).hexdigest()
        allg = [None] * world
        torch.distributed.all_gather_object(allg, dig)
        replicas = {"identical": len(set(allg)) == 1, "digests": sorted({d[:16] for d in allg})}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            cpu = cpu_baseline(args, P_init, H, W, train=args.mode == "train")
            cpu["config1"] = cpu_config1()
        except Exception as e:  # report, never fail the bench on the CPU leg
            cpu = {"error": repr(e)}

    # The secondary legs never cost the headline line: an exception (e.g. out of memory)
    # is recorded in the leg's own field and the JSON line is still printed.  Under N > 1
    # the ranks agree on each leg's outcome (a MIN all-reduce of an ok flag) before the
    # next leg's collectives, so one rank's failure marks the leg failed on every rank
    # instead of leaving the others blocked in a collective.  A leg's allocations (the
    # part that can fail on one rank alone) come before its first collective, where it
    # calls agree(ok) itself.
    def agree(ok):
        if world > 1:
            f = torch.tensor([1.0 if ok else 0.0], device="cuda")
            torch.distributed.all_reduce(f, op=torch.distributed.ReduceOp.MIN)
            if f.item() < 1.0 and ok:
                raise RuntimeError("leg failed on another rank")
        return ok

    def guarded(fn, *a):
        ok = True
        try:
            res = fn(*a)
        except Exception as e:
            ok = False
            import traceback
            traceback.print_exc()
            res = {"error": repr(e)[:500]}
        finally:
            timer.on = False
            timer.rec = []
            C.clear_session()
            torch.cuda.empty_cache()
        try:
            agree(ok)
        except RuntimeError:  # this rank's leg succeeded, another rank's failed: the leg failed
            res = {"error": "leg failed on another rank"}
        return res

    # configs[1]: fp32 inference leg (b8 1080p, BN moving stats), same ranks, weak
    infer = ns = k4 = f32t = None
    if args.mode == "train" and (args.infer_batch > 0 or args.k4_batch > 0 or args.ns_batch > 0
                                 or args.f32_train_batch > 0):
        del eng, model, x, t, losses
        timer.rec = []
        C.clear_session()
        torch.cuda.empty_cache()
    if args.mode == "train" and args.infer_batch > 0:
        infer = guarded(infer_leg, args, rank, world, timer, barrier, agree, P_init, H, W, args.infer_batch, True)
    # north star: fp32 conv2d forward at 1080p batch 32 (BASELINE.json "Target: >=40% of fp32 MFMA peak")
    if args.mode == "train" and args.ns_batch > 0:
        ns = guarded(infer_leg, args, rank, world, timer, barrier, agree, P_init, H, W, args.ns_batch, False)
    # configs[4]: 4K training (b8 per GPU = global 64 on 8 GPUs), DP when N > 1
    if args.mode == "train" and args.k4_batch > 0:
        k4 = guarded(k4_leg, args, rank, world, timer, barrier, agree, cpu)
    # fp32 training (the reference's precision; the drop-in default dtype of U_net)
    if args.mode == "train" and args.f32_train_batch > 0:
        f32t = guarded(f32_train_leg, args, rank, world, timer, barrier, agree, cpu)

    if rank == 0:
        res = "1080p" if (args.height, args.width) == (1080, 1920) else f"{args.width}x{args.height}"
        metric = f"{res} SDR->HDR frames/sec (fwd+bwd)" if args.mode == "train" else f"{res} SDR->HDR frames/sec (fwd)"
        line = {"metric": metric, "value": round(fps, 3), "unit": "frames/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "bf16" if args.dtype == "bfloat16" else "f32", "data": "synthetic",
                "config": {"workload": f"U-Net (model.py:204) {args.mode} step, {args.width}x{args.height} "
                                       f"frames padded to {W}x{H}, {B} frames/GPU",
                           "global_batch": B * world, "frame": [args.height, args.width],
                           "padded": [H, W], "parallelism": f"dp{world}",
                           "gflop_per_frame": round(step_flops / B / 1e9, 1)},
                "roofline": roof, "cpu_baseline": cpu}
        if exposed is not None:
            line["allreduce_exposed"] = exposed
        if replicas is not None:
            line["replicas"] = replicas
        if infer is not None:
            line["fp32_infer"] = infer
        if ns is not None:
            cb = (infer or {}).get("cpu_baseline") if isinstance(infer, dict) else None
            if isinstance(ns, dict) and ns.get("cpu_baseline") is None and cb and "value" in cb:
                # the oracle's fp32 inference rate is per frame, whatever the GPU batch: the
                # configs[1] leg's timing of the same forward, on the same host in this run
                ns["cpu_baseline"] = dict(cb, sample=cb.get("sample", "") + "; the fp32_infer leg's timing "
                                          "(frames/s of the same per-frame forward; the batch is a GPU-side choice)")
            line["fp32_infer_b32"] = ns
        if k4 is not None:
            line["k4_train"] = k4
        if f32t is not None:
            line["fp32_train"] = f32t
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def infer_leg(args, rank, world, timer, barrier, agree, P_init, H, W, B, with_cpu):
    """BASELINE configs[1]: 1080p frames, batch B (8) per GPU, fp32, forward-only inference
    (predict.py:62 semantics: BN moving stats), through Model.predict's engine path with
    inputs resident in HBM.  Its own roofline (dominant kernel, HIP events) and CPU
    baseline (the oracle's fp32 forward).  With B = 32 it is the north star's
    "fp32 conv2d fwd at 1080p batch=32" point."""
    import torch
    import cnn_itmo_amd as C
    ok = False
    try:  # allocations before the first collective (see main's agree)
        with contextlib.redirect_stdout(io.StringIO()):
            m = C.U_net(input_size=(args.height, args.width, 3), pad=True, dtype="float32", seed=0, verbose=False)
        # non-trivial moving statistics (seeded), as a trained checkpoint would hold
        rng = np.random.default_rng(5)
        named = {}
        for k, v in m.named_weights().items():
            if k.endswith("/moving_mean"):
                named[k] = rng.uniform(0.0, 0.5, v.shape).astype(np.float32)
            elif k.endswith("/moving_variance"):
                named[k] = rng.uniform(0.5, 2.0, v.shape).astype(np.float32)
        m.set_named_weights(named)
        P = m.named_weights() if rank == 0 else None
        eng = m._engine()
        torch.cuda.reset_peak_memory_stats()
        g = torch.Generator(device="cuda")
        g.manual_seed(77 + 7919 * rank)
        x = torch.randint(0, 256, (B, args.height, args.width, 3), generator=g, device="cuda",
                          dtype=torch.uint8).float() / 255.0
        yhat = torch.empty(B, args.height, args.width, 3, device="cuda", dtype=torch.float32)
        ok = True
    finally:
        agree(ok)

    def step():
        eng.predict_into(x, yhat)  # Model.predict's path: the head is computed every step

    def timed(n):
        barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        return el.item()

    for _ in range(max(1, min(args.warmup, 3) if B > 8 else args.warmup)):
        step()
    k = max(args.steps, 5) if B <= 8 else max(3, min(args.steps, 5))
    elapsed = timed(k)
    timer.reset()
    timer.on = True
    k2 = min(k, 10)
    elapsed2 = timed(k2)
    timer.on = False
    agg = timer.summary()
    roof, step_flops = _roofline(agg, k2, elapsed2, F32_PEAK_TF, _shape("infer", args.height, args.width, B, "float32"))
    roof["timed_pass_ms_per_step"] = round(elapsed2 / k2 * 1e3, 2)
    # the whole forward's conv FLOPs over its conv time: the north star's "% of fp32 MFMA peak on conv2d fwd"
    conv_ms = sum(v[2] for v in agg.values()) / k2
    roof["conv_fwd_tflops_all_layers"] = round(step_flops / (conv_ms * 1e-3) / 1e12, 2)
    roof["conv_fwd_frac_all_layers"] = round(step_flops / (conv_ms * 1e-3) / 1e12 / F32_PEAK_TF, 4)
    what = "BASELINE configs[1]" if B == 8 else "north star: fp32 conv2d fwd at 1080p batch 32"
    out = {"metric": "1080p SDR->HDR frames/sec (fwd, inference)", "value": round(B * world * k / elapsed, 3),
           "unit": "frames/s", "dtype": "f32", "steps": k, "ms_per_step": round(elapsed / k * 1e3, 2),
           "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
           "config": {"workload": f"U-Net inference forward, {args.width}x{args.height} frames padded to "
                                  f"{W}x{H}, {B} frames/GPU ({what})", "global_batch": B * world,
                      "gflop_per_frame": round(step_flops / B / 1e9, 1)},
           "roofline": roof, "cpu_baseline": None}
    if rank == 0:
        _print_agg(agg, f"infer b{B}")
        _print_detail(timer.detail(), k2, f"infer b{B}")
        if world == 1 and not args.no_cpu and with_cpu:
            try:
                out["cpu_baseline"] = cpu_baseline(args, P, H, W, train=False)
            except Exception as e:
                out["cpu_baseline"] = {"error": repr(e)}
    del eng, m, x, yhat
    return out


def _shape(mode, h, w, b, dtype):
    """Key of a profiled workload in profiles/pmc_traffic.json's _meta.shapes."""
    return f"{mode} {h}x{w} b{b} {dtype}"


def train_leg(args, rank, world, timer, barrier, agree, cpu_1080, Hk, Wk, B, dtype, steps, warmup, label):
    """A secondary training leg (fwd+bwd+RMSprop, DP over the same ranks when N > 1) with
    the headline's two passes: K timed steps without instrumentation, then min(K, 10)
    steps with every conv launch bracketed by HIP events (roofline of the dominant
    kernel, PMC traffic when the profiled shape matches).  cpu_baseline: the headline
    leg's oracle training step (one 960x544 crop, same run; the oracle computes in fp32)
    scaled to this frame size by pixel count."""
    import torch
    import cnn_itmo_amd as C
    ok = False
    try:  # everything that can fail alone (allocation) happens before the first collective
        with contextlib.redirect_stdout(io.StringIO()):
            m = C.U_net(input_size=(Hk, Wk, 3), pad=True, dtype=dtype, seed=0, verbose=False)
        eng = m._engine()
        g = torch.Generator(device="cuda")
        g.manual_seed(4321 + 7919 * rank)
        x = torch.randint(0, 256, (B, Hk, Wk, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
        t = torch.randint(0, 256, (B, Hk, Wk, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
        ok = True
    finally:
        agree(ok)
    dp = None
    if world > 1:
        m.distribute(bucket_mb=args.bucket_mb)
        dp = m._dp
    opt = m.optimizer
    torch.cuda.reset_peak_memory_stats()

    def step(i):
        kw = dict(seed=i * world + rank, lr=opt.lr, rho=opt.rho, eps=opt.epsilon)
        if dp is not None:
            kw.update(sync=dp.finish, grad_scale=dp.grad_scale)
        return eng.train_step(x, t, **kw)

    def timed(n, first):
        barrier()
        t0 = time.perf_counter()
        for i in range(n):
            out = step(first + i)
        barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        if world > 1:
            torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
        return el.item(), out

    for i in range(max(1, warmup)):
        step(i)
    k = max(1, steps)
    elapsed, out = timed(k, 100)
    loss = out.cpu().numpy().tolist() if out is not None else None
    timer.reset()
    timer.on = True
    k2 = max(1, min(k, 10))
    elapsed2, _ = timed(k2, 200)
    timer.on = False
    agg = timer.summary()
    Hp = -(-Hk // 16) * 16
    peak = BF16_PEAK_TF if dtype == "bfloat16" else F32_PEAK_TF
    roof, step_flops = _roofline(agg, k2, elapsed2, peak, _shape("train", Hk, Wk, B, dtype))
    roof["timed_pass_ms_per_step"] = round(elapsed2 / k2 * 1e3, 2)
    if rank == 0:
        _print_agg(agg, label)
        _print_detail(timer.detail(), k2, label)
    res_name = "4K" if (Hk, Wk) == (2160, 3840) else ("1080p" if (Hk, Wk) == (1080, 1920) else f"{Wk}x{Hk}")
    res = {"metric": f"{res_name} SDR->HDR frames/sec (fwd+bwd)", "value": round(B * world * k / elapsed, 3),
           "unit": "frames/s", "dtype": "bf16" if dtype == "bfloat16" else "f32", "steps": k, "warmup": max(1, warmup),
           "ms_per_step": round(elapsed / k * 1e3, 2),
           "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1), "last_loss_acc": loss,
           "config": {"workload": f"U-Net train step, {Wk}x{Hk} frames padded to {Wk}x{Hp}, {B} frames/GPU ({label})",
                      "global_batch": B * world, "parallelism": f"dp{world}",
                      "gflop_per_frame": round(step_flops / B / 1e9, 1)},
           "roofline": roof, "cpu_baseline": None}
    if cpu_1080 and "value" in cpu_1080:
        sc = (1920.0 * cpu_1080["padded_h"]) / (Wk * Hp)  # 1080p-frame equivalents -> these frames
        res["cpu_baseline"] = {"value": cpu_1080["value"] * sc, "unit": f"{res_name} frames/s (fwd+bwd, fp32)",
                               "cores": cpu_1080["cores"], "kind": cpu_1080["kind"],
                               "sample": cpu_1080["sample"] + f"; the same timing scaled to a {Wk}x{Hp} frame "
                                                              f"by pixel count (x{sc:.4f})",
                               "seconds": cpu_1080["seconds"], "threads_note": cpu_1080.get("threads_note")}
    del eng, m, x, t
    return res


def k4_leg(args, rank, world, timer, barrier, agree, cpu_1080):
    """BASELINE configs[4]: 3840x2160 frames, bf16, fwd+bwd+RMSprop, k4_batch frames per
    GPU (8 = global 64 on 8 GPUs).  The activations are not tiled: at 8 frames per GPU
    the step's working set fits one GPU's HBM (peak_mem_gib), so the frame is processed
    whole, which keeps every pixel's receptive field exact."""
    return train_leg(args, rank, world, timer, barrier, agree, cpu_1080, 2160, 3840, args.k4_batch, "bfloat16",
                     args.k4_steps, args.k4_warmup, "BASELINE configs[4]; whole frames, no spatial tiling needed")


def f32_train_leg(args, rank, world, timer, barrier, agree, cpu_1080):
    """The reference's own training precision (Keras fp32, main.py:126-132) at 1080p:
    fp32 storage and fp32 MFMA (16x16x4 f32), f32_train_batch frames per GPU."""
    return train_leg(args, rank, world, timer, barrier, agree, cpu_1080, args.height, args.width,
                     args.f32_train_batch, "float32", args.f32_train_steps, args.f32_train_warmup,
                     "fp32 training, main.py:126-132")


if __name__ == "__main__":
    main()
