"""Data parallelism: one process per GPU, batch sharded across ranks, weight
gradients all-reduced with RCCL (torch ``nccl`` backend == RCCL on ROCm) over xGMI.

The reference is single-GPU; this is the north star's
new DP path, reached from the reference's own training call
``model.fit_generator(...)`` (main.py:126-132) through
``Model.fit_generator(..., distributed=True)`` / ``Model.distribute()``.

Design for MI355X's point-to-point xGMI: the 11.16 M fp32 gradients (44.6 MB)
are split into a handful of large contiguous buckets of the flat gradient
buffer; because the engine lays parameters out in reverse stage order, backward
fills the buffer front to back and each bucket is launched (async, on RCCL's
stream, ordered after the producing kernels by torch's stream events) the
moment its last gradient is written -- overlapping the ring all-reduce with the
remaining backward.  Averaging is folded into the RMSprop kernel
(grad_scale = 1/world).

BatchNorm: the batch statistics that normalise a replica's activations are the
replica's own (Keras multi-GPU replication semantics).  The MOVING
statistics are **averaged over ranks every step**: right after the forward pass
(which updates them from the replica's batch) one async all-reduce of the
7,808-float moving-stat buffer is launched, it overlaps the backward, and
``finish()`` scales it by 1/world.  Since every rank starts from the same moving
stats (``broadcast_state``), the result is
``m <- momentum*m + (1-momentum)*mean_over_ranks(batch statistic)``, identical
on every rank, so a checkpoint written by any rank holds the same values.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _force():
    """CNNITMO_DIST_FORCE=1: run the collectives even in a one-rank group (a box with
    one GPU can then execute the RCCL path end to end: tools/rccl_world1.py)."""
    return os.environ.get("CNNITMO_DIST_FORCE") == "1"


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
    if (world > 1 or _force()) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def rank_world(group=None):
    """(rank, world) of the default (or given) process group; (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


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
    """Launches one async all-reduce per bucket as soon as backward has written it,
    plus (when given) one async all-reduce of the BN moving statistics right after
    the forward pass."""

    def __init__(self, grads, stage_ranges, bucket_mb=16.0, group=None, stats=None):
        self.grads = grads
        self.stats = stats
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.collect = self.world > 1 or (_force() and dist.is_initialized())
        order = sorted((r for r in stage_ranges if r[1] > r[0]), key=lambda r: r[0])
        self.buckets = make_buckets(order, int(bucket_mb * (1 << 20) / 4))
        self.timing = False      # record the compute stream's exposed wait in finish()
        self._events = []        # (ev_before_wait, ev_after_wait) per finish()
        self.reset()

    def reset(self):
        self.next = 0
        self.ready = 0
        self.works = []
        self.stat_work = None

    def _launch(self, lo, hi):
        if self.collect:
            self.works.append(dist.all_reduce(self.grads[lo:hi], group=self.group, async_op=True))

    def on_forward(self):
        """Engine callback after the forward pass: the moving statistics are final."""
        if self.collect and self.stats is not None and self.stats.numel():
            self.stat_work = dist.all_reduce(self.stats, group=self.group, async_op=True)

    def hook(self, lo, hi):
        """Engine callback: gradients [lo, hi) are enqueued (backward order)."""
        self.ready = max(self.ready, hi)
        while self.next < len(self.buckets) and self.buckets[self.next][1] <= self.ready:
            self._launch(*self.buckets[self.next])
            self.next += 1

    def finish(self):
        """Launch what is left, then make the current stream wait for every bucket
        (and the moving-stat average)."""
        while self.next < len(self.buckets):
            self._launch(*self.buckets[self.next])
            self.next += 1
        ev = None
        if self.timing and self.grads.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for w in self.works:
            w.wait()
        if self.stat_work is not None:
            self.stat_work.wait()
            self.stats.mul_(1.0 / self.world)
        if ev is not None:
            ev[1].record()
            self._events.append(ev)
        self.reset()

    def exposed_ms(self, clear=True):
        """Total time the compute stream spent waiting for the collectives in finish()
        (i.e. the all-reduce time NOT hidden behind backward), over the recorded steps."""
        tot = sum(a.elapsed_time(b) for a, b in self._events)
        n = len(self._events)
        if clear:
            self._events = []
        return tot, n

    @property
    def grad_scale(self):
        return 1.0 / self.world


def broadcast_state(engine, src=0, group=None):
    """DDP-style start: every rank takes rank `src`'s parameters, moving statistics,
    RMSprop accumulators and step counter."""
    for t in (engine.params, engine.bufs, engine.accum):
        dist.broadcast(t, src, group=group)
    step = torch.tensor([engine.step], dtype=torch.float64, device=engine.params.device)
    dist.broadcast(step, src, group=group)
    engine.step = int(step.item())
    engine.weights_dirty = True


def attach(engine, bucket_mb=16.0, group=None, broadcast=True):
    """Wire a GradBucketer into an Engine; returns it.  Use
    ``engine.train_step(..., sync=b.finish, grad_scale=b.grad_scale)``."""
    if broadcast and dist.is_initialized() and (dist.get_world_size(group) > 1 or _force()):
        broadcast_state(engine, group=group)
    b = GradBucketer(engine.grads, engine.stage_goff[::-1], bucket_mb, group, stats=engine.bufs)
    engine.grad_hook = b.hook
    engine.fwd_hook = b.on_forward
    return b
