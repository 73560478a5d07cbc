"""MultiWorkerMirroredStrategy: synchronous data parallelism over tfk_comm -- the runtime's own
RCCL communicator on GPUs (parallel/tfk_comm.py, csrc/bindings/comm.cpp), torch.distributed gloo
on the CPU tier.

MI355X design: gradients live in ONE flat f32 arena buffer laid out in backward-completion order,
so a bucket is a contiguous slice -> one ``all_reduce`` per bucket with no flatten copies. Buckets
are launched the moment the backward pass has written their last gradient (executor readiness
callbacks), so ring all-reduce over xGMI overlaps the remaining backward compute; RCCL runs on the
communicator's high-priority comm stream (forked at launch from the compute stream AND the
side streams that produced weight gradients, runtime/streams.py producers()) and the compute
stream only waits on it right before the optimizer -- the input-gradient chain never stalls behind
queued weight gradients at a bucket launch. Under hipGraph capture those forks/joins are
graph edges: the captured step (forward, backward, bucket all-reduces, optimizer) is the step that
runs at every world size.

* Launch order is the bucket order on every rank (a bucket that completes early waits for its
  predecessors), so all ranks issue the same collective sequence whatever the readiness callbacks
  do -- a mismatched order would pair different buckets in the ring and hang or corrupt.
* The default wire is f32 (RCCL sums exactly what TF's f32 gradient aggregation sums).
  ``comm_dtype=torch.bfloat16`` (opt-in, like TF's CommunicationOptions) puts bf16 on the wire:
  the bucket is packed f32->bf16 by a HIP
  cast kernel on the comm stream (after its producer waits), all-reduced in bf16 (half the
  xGMI bytes of f32: 51 MB instead of 102 MB per ResNet-50 step) and unpacked into the f32 arena
  right after the wait; the 1/world mean stays in the fused optimizer's grad_scale.
* Bucket size default 32 MiB of f32 gradient: large enough to amortise RCCL launch/latency on the
  7x153 GB/s point-to-point xGMI mesh, small enough that the last bucket's exposed tail is short.
* ``force=True`` runs the collectives even with world size 1 (exercises the RCCL path -- and its
  hipGraph capture -- on a single-GPU box).
* Everything here is hipGraph-capturable: no host synchronisation, all buffers pre-allocated.
"""
from __future__ import annotations

import torch

from ..runtime.arena import ParamArena
from . import tfk_comm

_COMM_DTYPES = {"f32": torch.float32, "fp32": torch.float32, "float32": torch.float32,
                "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


def comm_dtype_of(x) -> torch.dtype:
    if isinstance(x, torch.dtype):
        if x not in (torch.float32, torch.bfloat16):
            raise ValueError(f"MWMS comm_dtype must be float32 or bfloat16, got {x}")
        return x
    try:
        return _COMM_DTYPES[str(x).lower()]
    except KeyError:
        raise ValueError(f"MWMS comm_dtype must be f32|bf16, got {x!r}") from None


class Bucket:
    __slots__ = ("start", "end", "nparams", "pending", "work", "launched")

    def __init__(self, start, end, nparams):
        self.start, self.end, self.nparams = start, end, nparams
        self.pending = nparams
        self.work = None
        self.launched = False


class MultiWorkerMirroredStrategy:
    name = "mwms"

    def __init__(self, arena: ParamArena, comm=None, bucket_mb: float = 32.0, comm_dtype=torch.float32,
                 force: bool = False):
        self.arena = arena
        self.comm = comm if comm is not None else tfk_comm.world()
        inited = self.comm is not None
        self.world = self.comm.world if inited else 1
        self.rank = self.comm.rank if inited else 0
        self.comm_dtype = comm_dtype_of(comm_dtype)
        self.buckets: list[Bucket] = []
        self.bucket_of: dict[int, Bucket] = {}
        self._build(int(bucket_mb * (1 << 20)) // 4)
        self.enabled = self.world > 1 or (force and inited)
        self._next = 0  # index of the next bucket to launch (in-order launch)
        self.wire = None
        if self.enabled and self.comm_dtype != torch.float32:
            self.wire = torch.empty(arena.numel, dtype=self.comm_dtype, device=arena.grad.device)
        if self.enabled:
            arena.on_grad_ready(self._on_ready)

    def _build(self, elems_per_bucket: int):
        params = sorted(self.arena.params, key=lambda p: p.offset)
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

    def wire_bytes(self) -> int:
        """Bytes one rank contributes to the gradient all-reduce per step."""
        return sum(b.end - b.start for b in self.buckets) * (2 if self.comm_dtype == torch.bfloat16 else 4)

    # ------------------------------------------------------------------ per step
    def begin_step(self):
        for b in self.buckets:
            b.pending, b.work, b.launched = b.nparams, None, False
        self._next = 0

    def _on_ready(self, p):
        b = self.bucket_of.get(p.index)
        if b is None:
            return
        b.pending -= 1
        # launch every leading bucket whose gradients are complete, in bucket order
        while self._next < len(self.buckets) and self.buckets[self._next].pending <= 0:
            self._launch(self.buckets[self._next])
            self._next += 1

    def _launch(self, b: Bucket):
        b.launched = True
        from ..runtime import streams
        # the bucket may hold weight gradients produced on the side streams: the COMM stream waits
        # for them (and for the compute stream); the compute stream's input-gradient chain does not
        deps = streams.producers()
        view = self.arena.grad[b.start:b.end]
        pre = None
        if self.wire is not None:
            from ..ops.optim import cast_f32_bf16
            w = self.wire[b.start:b.end]
            pre = (lambda v=view, w=w: cast_f32_bf16(v, w))  # packed on the comm stream
            view = w
        b.work = self.comm.all_reduce(view, async_op=True, deps=deps, pre=pre)

    def finish_step(self):
        """Launch stragglers (in order), wait for every bucket (compute stream waits on the RCCL
        stream), unpack bf16 wire buckets into the f32 arena."""
        if not self.enabled:
            return
        while self._next < len(self.buckets):
            self._launch(self.buckets[self._next])
            self._next += 1
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if self.wire is not None:
                    from ..ops.optim import cast_bf16_f32
                    cast_bf16_f32(self.wire[b.start:b.end], self.arena.grad[b.start:b.end])

    def configure_optimizer(self, opt) -> None:
        opt.grad_scale = 1.0 / self.world

    # ------------------------------------------------------------------ state sync
    def broadcast_parameters(self, src: int = 0):
        """Chief's master weights + non-trainable buffers everywhere: the arena is one broadcast,
        the buffers (BN moving statistics, ...) are coalesced into one flat tensor per dtype."""
        if not self.enabled:
            return
        self.comm.broadcast(self.arena.master, src)
        by_dtype: dict = {}
        for b in self.arena.buffers:
            by_dtype.setdefault((b.tensor.dtype, b.tensor.device), []).append(b.tensor)
        for ts in by_dtype.values():
            flat = torch.cat([t.reshape(-1) for t in ts])
            self.comm.broadcast(flat, src)
            o = 0
            for t in ts:
                t.copy_(flat[o:o + t.numel()].view_as(t))
                o += t.numel()
        self.arena.refresh_compute()

    def all_reduce_metrics(self, t: torch.Tensor) -> torch.Tensor:
        if self.enabled:
            self.comm.all_reduce(t)
        return t
