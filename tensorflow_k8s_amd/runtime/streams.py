"""Side HIP stream for weight-gradient GEMMs.

A conv's weight gradient dW = dY^T im2col(X) and its input gradient dX = dY W^T both depend only on
dY, so the weight gradients run on a second stream, concurrent with the main stream's serial
input-gradient chain (dgrad GEMMs, BatchNorm backward passes). On MI355X the late ResNet stages
issue dgrad grids far smaller than 256 CUs x occupancy, so the concurrent wgrad grids fill the idle
CUs. Under hipGraph capture the fork (side waits on the capture stream) and the join become graph
edges.

Ordering contract:
* ``run_wgrad(fn, *tensors)`` forks after everything queued on the current stream and keeps
  ``tensors`` (what fn reads) alive until the next ``join()``. The caching allocator may otherwise
  hand their memory to later main-stream kernels while the side stream still reads it.
* ``producers()``: issue the queued weight gradients and return the side streams forked since the
  last join. Gradient-bucket collectives (MWMS all-reduce, PS reduce) make THEIR comm stream wait
  on these plus the current stream -- a bucket mixes gradients from both -- so the main stream's
  input-gradient chain never waits for queued weight gradients at a bucket launch.
* ``sync()``: the current stream waits for all side-stream work.
* ``join()``: sync plus release the kept tensors. Models call it at the end of backward, before the
  optimizer reads ``arena.grad``.

Mode (TFK_CONCURRENT_WGRAD): "auto" (default) forks only while a hipGraph is being captured, "1"
always, "0" never. Measured on MI355X (ResNet-50 bs256, same box):
* hipGraph replay: 25.90 ms/step with the side stream vs 26.48 without.
* eager steps (the multi-GPU path), forced RCCL: 26.91 vs 26.11. The per-layer fork/join adds host
  work that makes the eager step launch-bound.
"""
from __future__ import annotations

import os

import torch

MODE = os.environ.get("TFK_CONCURRENT_WGRAD", "auto")
# side streams used round-robin (each with its own split-K workspace slot): a weight gradient's slab
# reduce then overlaps the next weight gradient's GEMM. Measured (ResNet-50 bs256, same box):
# 1 -> 25.64 ms, 2 -> 25.41 ms, 3 -> 25.76 ms; re-measured with the halved side-stream wgrad fill
# (round 5, alternating): 1 -> 21.85 / 21.95, 2 -> 21.64 / 21.73 / 21.71, 3 -> 22.20 / 22.16 / 22.18
NSIDE = int(os.environ.get("TFK_NSIDE", "2"))
_side: dict[tuple[int, int], torch.cuda.Stream] = {}
_keep: list[torch.Tensor] = []
_rr = 0


def _stream(dev: torch.device) -> tuple[int, torch.cuda.Stream]:
    global _rr
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    k = _rr % max(1, NSIDE)
    _rr += 1
    s = _side.get((idx, k))
    if s is None:
        s = _side[(idx, k)] = torch.cuda.Stream(device=idx)
    return k, s


# Weight-gradient forks per residual block instead of per conv (A/B switch, tools): under hipGraph
# each fork/join is a cross-queue edge of the replayed graph, and the trace shows ~10-12 us with no
# kernel running at each (88 gaps, 0.54 ms per ResNet-50 step). DEFER queues the deferrable weight
# gradients and flush() issues them behind ONE fork (the model calls it at the end of each block).
DEFER = True
# flush() issues the queue on every FLUSH_EVERY-th call (1: one fork per residual block)
FLUSH_EVERY = 1
_pending: list = []
_flushes = 0
_used: dict[int, torch.cuda.Stream] = {}  # side streams forked since the last join (by id)


def _concurrent(tensors) -> bool:
    return bool(tensors and tensors[0].is_cuda and MODE != "0"
                and (MODE == "1" or torch.cuda.is_current_stream_capturing()))


def _fork(items) -> None:
    from ..ops import _lib
    dev = items[0][1][0].device
    main = torch.cuda.current_stream(dev)
    k, side = _stream(dev)
    side.wait_stream(main)
    _used[id(side)] = side
    prev = _lib.WGRAD_SLOT
    _lib.WGRAD_SLOT, _lib.ON_SIDE_STREAM = f"splitk_wgrad{k}", True
    try:
        with torch.cuda.stream(side):
            for fn, _ in items:
                fn()
    finally:
        _lib.WGRAD_SLOT, _lib.ON_SIDE_STREAM = prev, False
    for _, tensors in items:
        _keep.extend(tensors)


def run_wgrad(fn, *tensors: torch.Tensor, deferrable: bool = False) -> None:
    """Run fn() (weight-gradient GEMMs reading `tensors`) on the side stream. deferrable: with DEFER,
    queue it for the next flush() instead of forking now."""
    if not _concurrent(tensors):
        fn()
        return
    if DEFER and deferrable:
        _pending.append((fn, tensors))
        return
    _fork([(fn, tensors)])


def flush(force: bool = False) -> None:
    """Issue the queued (deferred) weight gradients behind one fork (every FLUSH_EVERY-th call,
    or now with force)."""
    global _flushes
    _flushes += 1
    if not force and _flushes % max(1, FLUSH_EVERY):
        return
    if _pending:
        items = list(_pending)
        _pending.clear()
        _fork(items)


def producers() -> list:
    """Issue the queued weight gradients; return the side streams (forked since the last join) that a
    consumer of arena.grad on ANOTHER stream must wait on. The current stream is not joined."""
    flush(force=True)
    return list(_used.values())


def sync() -> None:
    """The current stream waits for every weight gradient queued on the side stream."""
    flush(force=True)
    if _side and torch.cuda.is_available():
        main = torch.cuda.current_stream()
        for s in _side.values():
            main.wait_stream(s)


def reset() -> None:
    """Drop every queued (unissued) weight gradient and kept tensor: after a step capture that
    raised mid-backward, the queue holds closures over the dropped graph's tensors, which must
    never run in a later step (the caller synchronizes the device first)."""
    global _flushes
    _pending.clear()
    _keep.clear()
    _used.clear()
    _flushes = 0


def join() -> None:
    """sync() + release the tensors the side-stream work read."""
    sync()
    _keep.clear()
    _used.clear()
