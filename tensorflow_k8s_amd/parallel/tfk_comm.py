"""tfk_comm: the communication layer the strategies (MWMS, collective PS) run on.

Two implementations of one small interface:

* ``RcclComm`` (GPU): the runtime's own RCCL communicator (``csrc/bindings/comm.cpp``, linked against
  the librccl.so torch loads). Bootstrap is TF-style: the chief draws an ``ncclUniqueId`` and
  publishes it in the job's TCP store (the store on the chief's tfPort that ``cluster.make_store``
  opens), every rank reads it and calls ``ncclCommInitRank``. Collectives run on a dedicated
  high-priority comm stream that is forked from / joined to the caller's stream with events, so
  (a) gradient buckets overlap the rest of backward, and (b) under hipGraph capture the fork, the
  RCCL kernels and the join become graph nodes and edges -- the whole data-parallel step replays
  as one graph at any world size. ``abort()`` is ``ncclCommAbort`` (the watchdog calls it).
* ``TorchDistComm`` (CPU tier, tests, CPU parameter servers): the same calls over torch.distributed's
  gloo backend; handles wrap gloo work objects.

Async calls return a handle whose ``wait()`` orders the caller's current stream after the
collective (GPU: a stream-event wait, no host block; CPU: blocks).
"""
from __future__ import annotations

import contextlib
import datetime
import os
import threading
import weakref

import torch

_LIVE: "weakref.WeakSet[RcclComm]" = weakref.WeakSet()
_LIVE_LOCK = threading.Lock()


def abort_all() -> int:
    """ncclCommAbort every live communicator of this process (watchdog path). Returns the count."""
    with _LIVE_LOCK:
        comms = list(_LIVE)
    n = 0
    for c in comms:
        try:
            if c.abort():
                n += 1
        except Exception:  # pragma: no cover - the process is exiting anyway
            pass
    return n


def async_errors() -> str:
    """The first asynchronous RCCL error of any live communicator ("" while all are healthy); the
    step watchdog polls this every tick (ncclCommGetAsyncError is thread-safe)."""
    with _LIVE_LOCK:
        comms = list(_LIVE)
    for c in comms:
        try:
            e = c.async_error()
        except Exception as ex:  # pragma: no cover - a broken communicator is an error too
            e = str(ex)
        if e:
            return f"{getattr(c, 'tag', '?')}: {e}"
    return ""


MIN_RCCL = 21800  # ncclCommSplit / ncclCommFinalize


def check_rccl_version(header: int, runtime: int) -> None:
    """The binding compiles against /opt/rocm's rccl.h but runs on the librccl torch loads: refuse a
    runtime of another major family, or one older than the entry points the binding calls."""
    if header // 10000 != runtime // 10000:
        raise RuntimeError(f"tfk_comm: librccl {runtime} is not the major family of rccl.h {header}")
    if runtime < MIN_RCCL:
        raise RuntimeError(f"tfk_comm: librccl {runtime} predates ncclCommSplit/ncclCommFinalize ({MIN_RCCL})")


def exchange_unique_id(store, rank: int, tag: str, make_uid, timeout_s: float = 300.0) -> bytes:
    """Rank 0 draws the communicator's unique id and publishes it under ``tfk_comm/<tag>/uid`` in the
    job store; every other rank waits for the key and reads it."""
    key = f"tfk_comm/{tag}/uid"
    if rank == 0:
        store.set(key, make_uid())
    else:
        store.wait([key], datetime.timedelta(seconds=timeout_s))
    return bytes(store.get(key))


class _StreamHandle:
    """Completion of an RCCL call on the comm stream; wait() = the caller's stream waits on it."""
    __slots__ = ("event",)

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)

    def is_completed(self) -> bool:
        return self.event.query()


class _WorkHandle:
    __slots__ = ("work",)

    def __init__(self, work):
        self.work = work

    def wait(self):
        if self.work is not None:
            self.work.wait()


class _Done:
    def wait(self):
        pass


_DONE = _Done()


# ------------------------------------------------------------------------------------------ RCCL
class RcclComm:
    backend = "rccl"

    def __init__(self, native, device: torch.device, tag: str = "world"):
        self._c = native
        self.device = device
        self.tag = tag
        self.rank, self.world = native.rank, native.size
        # comm stream: RCCL kernels of this communicator; priority -1 = high on ROCm, so bucket
        # all-reduces are not starved behind the backward grids queued on the compute stream
        self.stream = torch.cuda.Stream(device=device, priority=-1)
        self.store = None  # the job store the communicator was bootstrapped from (agreements)
        self._aborted = False
        with _LIVE_LOCK:
            _LIVE.add(self)

    # ------------------------------------------------------------------ bootstrap
    @classmethod
    def from_store(cls, store, rank: int, world: int, device: torch.device, tag: str = "world",
                   timeout_s: float = 300.0) -> "RcclComm":
        """Chief publishes the unique id under ``tfk_comm/<tag>/uid``; all ranks init."""
        from .. import _C
        check_rccl_version(_C.rccl_header_version(), _C.rccl_version())
        uid = exchange_unique_id(store, rank, tag, _C.rccl_unique_id, timeout_s)
        native = _C.RcclComm(uid, world, rank, device.index if device.index is not None else torch.cuda.current_device())
        c = cls(native, device, tag)
        c.store = store
        return c

    def split(self, ranks: list[int], tag: str) -> "RcclComm | None":
        """Sub-communicator over ``ranks`` (ncclCommSplit; every rank must call, in order)."""
        color = 0 if self.rank in ranks else -1
        key = sorted(ranks).index(self.rank) if self.rank in ranks else 0
        nc = self._c.split(color, key)
        if nc is None:
            return None
        c = RcclComm(nc, self.device, tag)
        c.store = self.store
        return c

    # ------------------------------------------------------------------ stream plumbing
    def _fork(self, deps=()):
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        for d in deps:
            self.stream.wait_stream(d)

    def _handle(self):
        ev = torch.cuda.Event()
        ev.record(self.stream)
        return _StreamHandle(ev)

    def _run(self, fn, async_op: bool, deps=(), pre=None):
        """deps: further producer streams the collective waits on (besides the caller's stream);
        pre: producer kernels (e.g. a wire-dtype pack) issued on the comm stream before it."""
        self._fork(deps)
        if pre is not None:
            with torch.cuda.stream(self.stream):
                pre()
        fn(self.stream.cuda_stream)
        h = self._handle()
        if async_op:
            return h
        h.wait()
        return None

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False, out: torch.Tensor | None = None,
                   deps=(), pre=None):
        o = t if out is None else out
        return self._run(lambda s: self._c.all_reduce(t, o, op, s), async_op, deps, pre)

    def reduce(self, t: torch.Tensor, root: int, op: str = "sum", async_op: bool = False, deps=(), pre=None):
        return self._run(lambda s: self._c.reduce(t, t, root, op, s), async_op, deps, pre)

    def broadcast(self, t: torch.Tensor, root: int, async_op: bool = False):
        return self._run(lambda s: self._c.broadcast(t, root, s), async_op)

    def all_gather(self, out: torch.Tensor, t: torch.Tensor, async_op: bool = False):
        return self._run(lambda s: self._c.all_gather(out, t, s), async_op)

    def reduce_scatter(self, out: torch.Tensor, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        return self._run(lambda s: self._c.reduce_scatter(out, t, op, s), async_op)

    def all_to_all(self, out: torch.Tensor, t: torch.Tensor, async_op: bool = False):
        return self._run(lambda s: self._c.all_to_all(out, t, s), async_op)

    def send(self, t: torch.Tensor, peer: int, async_op: bool = False):
        return self._run(lambda s: self._c.send(t, peer, s), async_op)

    def recv(self, t: torch.Tensor, peer: int, async_op: bool = False):
        return self._run(lambda s: self._c.recv(t, peer, s), async_op)

    @contextlib.contextmanager
    def group(self):
        """ncclGroupStart/End around a batch of point-to-point calls (PS push/pull), fused into one
        launch: ``with comm.group() as g: g.send(a, 1); g.recv(b, 1)`` then ``g.handle.wait()``."""
        from .. import _C
        self._fork()
        g = _RcclGroup(self)
        _C.rccl_group_start()
        try:
            yield g
        finally:
            _C.rccl_group_end()
        g.handle = self._handle()

    def barrier(self):
        x = torch.ones(1, dtype=torch.float32, device=self.device)
        self.all_reduce(x)
        torch.cuda.current_stream(self.device).synchronize()

    def async_error(self) -> str:
        return self._c.async_error()

    def abort(self) -> bool:
        if self._aborted:
            return False
        self._aborted = True
        self._c.abort()
        return True

    def destroy(self):
        # leave the live set FIRST: while ncclCommFinalize/Destroy runs (GIL released) the watchdog's
        # async-error poll must not read the communicator's own teardown as an RCCL failure
        with _LIVE_LOCK:
            _LIVE.discard(self)
        if not self._aborted:
            self._aborted = True
            self._c.destroy()


class _RcclGroup:
    def __init__(self, comm: RcclComm):
        self._comm, self.handle = comm, None

    def send(self, t, peer):
        self._comm._c.send(t, peer, self._comm.stream.cuda_stream)

    def recv(self, t, peer):
        self._comm._c.recv(t, peer, self._comm.stream.cuda_stream)


class _DistGroup:
    def __init__(self, comm: "TorchDistComm"):
        self._comm, self._works = comm, []
        self.handle = self

    def send(self, t, peer):
        self._works.append(self._comm.send(t, peer, async_op=True))

    def recv(self, t, peer):
        self._works.append(self._comm.recv(t, peer, async_op=True))

    def wait(self):
        for w in self._works:
            w.wait()
        self._works = []


# ------------------------------------------------------------------------------------------ gloo
class TorchDistComm:
    """CPU tier: a torch.distributed process group (gloo) behind the tfk_comm interface."""

    def __init__(self, group=None, store=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.store = store
        self.tag = "gloo"
        self.backend = str(dist.get_backend(group))
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device("cpu")
        self._global = {r: dist.get_global_rank(group, r) if group is not None else r for r in range(self.world)}

    _OPS = {"sum": "SUM", "max": "MAX", "min": "MIN", "prod": "PRODUCT", "avg": "AVG"}

    def _op(self, op):
        return getattr(self.dist.ReduceOp, self._OPS[op])

    def _w(self, work, async_op):
        return _WorkHandle(work) if async_op else None

    def split(self, ranks: list[int], tag: str) -> "TorchDistComm | None":
        g = self.dist.new_group([self._global[r] for r in sorted(ranks)])
        return TorchDistComm(g, self.store) if self.rank in ranks else None

    def all_reduce(self, t, op="sum", async_op=False, out=None, deps=(), pre=None):
        if pre is not None:
            pre()
        if out is not None and out.data_ptr() != t.data_ptr():
            out.copy_(t)
            t = out
        return self._w(self.dist.all_reduce(t, op=self._op(op), group=self.group, async_op=async_op), async_op)

    def reduce(self, t, root, op="sum", async_op=False, deps=(), pre=None):
        if pre is not None:
            pre()
        return self._w(self.dist.reduce(t, self._global[root], op=self._op(op), group=self.group, async_op=async_op),
                       async_op)

    def broadcast(self, t, root, async_op=False):
        return self._w(self.dist.broadcast(t, self._global[root], group=self.group, async_op=async_op), async_op)

    def all_gather(self, out, t, async_op=False):
        return self._w(self.dist.all_gather_into_tensor(out, t, group=self.group, async_op=async_op), async_op)

    def reduce_scatter(self, out, t, op="sum", async_op=False):
        # gloo has no reduce_scatter_tensor: all-reduce a copy and keep this rank's slice
        tmp = t.clone()
        self.dist.all_reduce(tmp, op=self._op(op), group=self.group)
        n = out.numel()
        out.copy_(tmp.reshape(-1)[self.rank * n:(self.rank + 1) * n].view_as(out))
        return _DONE if async_op else None

    def all_to_all(self, out, t, async_op=False):
        return self._w(self.dist.all_to_all_single(out, t, group=self.group, async_op=async_op), async_op)

    def send(self, t, peer, async_op=False):
        if async_op:
            return _WorkHandle(self.dist.isend(t, self._global[peer], group=self.group))
        self.dist.send(t, self._global[peer], group=self.group)

    def recv(self, t, peer, async_op=False):
        if async_op:
            return _WorkHandle(self.dist.irecv(t, self._global[peer], group=self.group))
        self.dist.recv(t, self._global[peer], group=self.group)

    @contextlib.contextmanager
    def group(self):
        yield _DistGroup(self)

    def barrier(self):
        self.dist.barrier(group=self.group)

    def async_error(self) -> str:
        return ""

    def abort(self) -> bool:
        return False

    def destroy(self):
        pass


# ------------------------------------------------------------------------------------------ setup
_WORLD = None


def world():
    """The process-wide training communicator: the one ``init`` created, else a wrapper of an
    already initialised torch.distributed default group (CPU tests), else None (single process)."""
    if _WORLD is not None:
        return _WORLD
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return TorchDistComm()
    return None


def set_world(c) -> None:
    global _WORLD
    _WORLD = c


def init(store, rank: int, world_size: int, device: torch.device, timeout_s: float = 300.0):
    """Create the world communicator for this process: RCCL for GPU ranks, gloo otherwise (the
    gloo process group is created on the same store). Returns it (also ``world()``)."""
    if device.type == "cuda":
        c = RcclComm.from_store(store, rank, world_size, device, "world", timeout_s)
    else:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group("gloo", store=store, rank=rank, world_size=world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s))
        c = TorchDistComm(store=store)
    set_world(c)
    return c


def env_store(rank: int, world_size: int, timeout_s: float = 300.0):
    """The launcher's TCP store (torchrun: MASTER_ADDR/MASTER_PORT, or the elastic agent's store when
    TORCHELASTIC_USE_AGENT_STORE is set), via torch's env:// rendezvous."""
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world_size,
                                       timeout=datetime.timedelta(seconds=timeout_s)))
    return store


def shutdown() -> None:
    """Orderly teardown of the world communicator (all ranks)."""
    global _WORLD
    c, _WORLD = _WORLD, None
    if c is not None:
        c.destroy()
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
