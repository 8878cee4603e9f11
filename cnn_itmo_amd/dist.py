"""Data parallelism: one process per GPU, batch sharded across ranks, weight
gradients all-reduced with RCCL (torch ``nccl`` backend == RCCL on ROCm) over xGMI.

The reference is single-GPU; this is the north star's
new DP path.  Design for MI355X's point-to-point xGMI: the 11.16 M fp32
gradients (44.6 MB) are split into a handful of large contiguous buckets of the
flat gradient buffer; because the engine lays parameters out in reverse stage
order, backward fills the buffer front to back and each bucket is launched
(async, on RCCL's stream, ordered after the producing kernels by torch's stream
events) the moment its last gradient is written -- overlapping the ring
all-reduce with the remaining backward.  BatchNorm statistics stay per replica
(Keras multi-GPU replication semantics), so no other collective is needed.
Averaging is folded into the RMSprop kernel (grad_scale = 1/world).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None):
    """Initialise the default process group from torchrun-style env vars.
    Returns (rank, world, local_rank)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (several ranks on one GPU): CNNITMO_DIST_BACKEND=gloo and
    # CNNITMO_DEVICE=<index> (every rank on that device)
    if os.environ.get("CNNITMO_DEVICE") is not None:
        local = int(os.environ["CNNITMO_DEVICE"])
    backend = backend or os.environ.get("CNNITMO_DIST_BACKEND") or None
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def make_buckets(stage_ranges, bucket_floats):
    """Greedy contiguous buckets over stage gradient ranges given in backward order
    (ascending offsets).  A bucket closes once it holds >= bucket_floats."""
    buckets = []
    lo = None
    hi = 0
    for a, b in stage_ranges:
        if b <= a:
            continue
        if lo is None:
            lo = a
        hi = b
        if hi - lo >= bucket_floats:
            buckets.append((lo, hi))
            lo = None
    if lo is not None:
        buckets.append((lo, hi))
    return buckets


class GradBucketer:
    """Launches one async all-reduce per bucket as soon as backward has written it."""

    def __init__(self, grads, stage_ranges, bucket_mb=16.0, group=None):
        self.grads = grads
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        order = sorted((r for r in stage_ranges if r[1] > r[0]), key=lambda r: r[0])
        self.buckets = make_buckets(order, int(bucket_mb * (1 << 20) / 4))
        self.reset()

    def reset(self):
        self.next = 0
        self.ready = 0
        self.works = []

    def _launch(self, lo, hi):
        if self.world > 1:
            self.works.append(dist.all_reduce(self.grads[lo:hi], group=self.group, async_op=True))

    def hook(self, lo, hi):
        """Engine callback: gradients [lo, hi) are enqueued (backward order)."""
        self.ready = max(self.ready, hi)
        while self.next < len(self.buckets) and self.buckets[self.next][1] <= self.ready:
            self._launch(*self.buckets[self.next])
            self.next += 1

    def finish(self):
        """Launch what is left, then make the current stream wait for every bucket."""
        while self.next < len(self.buckets):
            self._launch(*self.buckets[self.next])
            self.next += 1
        for w in self.works:
            w.wait()
        self.reset()

    @property
    def grad_scale(self):
        return 1.0 / self.world


def attach(engine, bucket_mb=16.0, group=None):
    """Wire a GradBucketer into an Engine; returns it.  Use
    ``engine.train_step(..., sync=b.finish, grad_scale=b.grad_scale)``."""
    b = GradBucketer(engine.grads, engine.stage_goff[::-1], bucket_mb, group)
    engine.grad_hook = b.hook
    return b
