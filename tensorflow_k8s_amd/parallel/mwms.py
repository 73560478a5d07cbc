"""MultiWorkerMirroredStrategy: synchronous data parallelism over RCCL (torch.distributed "nccl"
backend on ROCm) / gloo on CPU.

MI355X design: gradients live in ONE flat f32 arena buffer laid out in backward-completion order,
so a bucket is a contiguous slice -> one ``all_reduce`` per bucket with no flatten copies. Buckets
are launched the moment the backward pass has written their last gradient (executor readiness
callbacks), so ring all-reduce over xGMI overlaps the remaining backward compute; RCCL runs on its
own internal stream and the compute stream only waits on it right before the optimizer.
Bucket size default 32 MiB: large enough to amortise RCCL launch/latency on the 7x153 GB/s xGMI
mesh, small enough that the last bucket's exposed tail is short.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..runtime.arena import ParamArena


class Bucket:
    __slots__ = ("start", "end", "nparams", "pending", "work", "launched")

    def __init__(self, start, end, nparams):
        self.start, self.end, self.nparams = start, end, nparams
        self.pending = nparams
        self.work = None
        self.launched = False


class MultiWorkerMirroredStrategy:
    name = "mwms"

    def __init__(self, arena: ParamArena, group=None, bucket_mb: float = 32.0, comm_dtype: torch.dtype = torch.float32):
        self.arena = arena
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if self.world > 1 else 0
        self.comm_dtype = comm_dtype
        self.buckets: list[Bucket] = []
        self.bucket_of: dict[int, Bucket] = {}
        self._build(int(bucket_mb * (1 << 20)) // 4)
        self.enabled = self.world > 1
        if self.enabled:
            arena.on_grad_ready(self._on_ready)

    def _build(self, elems_per_bucket: int):
        params = sorted(self.arena.params, key=lambda p: p.offset)
        cur, start, n = [], None, 0
        regions = [self.arena.decay_region(), self.arena.nodecay_region()]
        for lo, hi in regions:
            grp = [p for p in params if lo <= p.offset < hi]
            cur, start = [], lo
            for p in grp:
                cur.append(p)
                end = p.offset + p.numel
                if end - start >= elems_per_bucket:
                    self._add(start, self._aligned_end(p, hi), cur)
                    cur, start = [], self._aligned_end(p, hi)
            if cur:
                self._add(start, hi, cur)

    def _aligned_end(self, p, hi):
        from ..runtime.arena import ALIGN
        return min(hi, p.offset + ((p.numel + ALIGN - 1) // ALIGN) * ALIGN)

    def _add(self, s, e, params):
        b = Bucket(s, e, len(params))
        self.buckets.append(b)
        for p in params:
            self.bucket_of[p.index] = b

    # ------------------------------------------------------------------ per step
    def begin_step(self):
        for b in self.buckets:
            b.pending, b.work, b.launched = b.nparams, None, False

    def _on_ready(self, p):
        b = self.bucket_of.get(p.index)
        if b is None:
            return
        b.pending -= 1
        if b.pending == 0 and not b.launched:
            self._launch(b)

    def _launch(self, b: Bucket):
        b.launched = True
        view = self.arena.grad[b.start:b.end]
        b.work = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish_step(self):
        """Launch stragglers, wait for every bucket (compute stream waits on the RCCL stream)."""
        if not self.enabled:
            return
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()

    def configure_optimizer(self, opt) -> None:
        opt.grad_scale = 1.0 / self.world

    # ------------------------------------------------------------------ state sync
    def broadcast_parameters(self, src: int = 0):
        if self.world <= 1:
            return
        dist.broadcast(self.arena.master, src, group=self.group)
        for b in self.arena.buffers:
            dist.broadcast(b.tensor, src, group=self.group)
        self.arena.refresh_compute()

    def all_reduce_metrics(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t
