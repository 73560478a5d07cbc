"""ParameterServerStrategy: variables sharded over "ps" tasks, gradients pushed by workers.

TF's ParameterServerStrategy (the reference's PS-style TFJobs, e.g. tf_cnn_benchmarks with
``--variable_update=parameter_server`` / examples/dist-mnist) places variables
on ps tasks; workers read them, compute gradients and send updates back, synchronously or
asynchronously. tfk equivalent:

* the flat parameter arena is split into ``len(ps)`` contiguous, ALIGN-aligned shards balanced by
  size; ps task s owns shard s: the f32 master copy plus the optimizer slots, and runs the
  optimizer for it (fused CPU path of ops.optim — ps tasks are CPU processes, as in TF);
* workers (one per GPU) run forward/backward on the device, copy each gradient shard to pinned
  host memory, push it to its owner and pull the updated shard back (gloo point-to-point over
  TCP; GPU<->GPU traffic between workers does not exist in this strategy);
* ``mode="sync"``: ps sums the pushes of all workers for step t, applies one update (mean
  gradient) and answers everyone -> identical parameters everywhere (TF SyncReplicasOptimizer);
  ``mode="async"``: ps applies each push as it arrives (Hogwild-style staleness, TF's default PS
  behaviour) and answers that worker only.

Two transports:
* ``transport="gloo"`` (ps tasks on CPU; sync or async): message protocol per (worker, shard):
  header int64[4] = [cmd, step, worker_rank, 0] then payload. cmd PUSH=1 (payload grad shard f32)
  -> reply shard f32; DONE=2; FETCH=3 (reply master + slots, for checkpoints); LOAD=4 (payload
  master + slots, restore); PULL=5 (reply master shard).
* ``transport="rccl"`` (ps tasks own a GPU, e.g. BASELINE's PS=2/worker=6 on one 8xMI355X node;
  sync only), bucketed and overlapped (``CollectivePlan``) on tfk_comm (the runtime's own RCCL
  communicator, parallel/tfk_comm.py; torch.distributed gloo on the CPU tier):
  - each shard is cut into parameter-aligned buckets (<= bucket_mb); every shard s has two
    sub-communicators (ncclCommSplit) over {its owner} + workers -- one for gradient ``reduce``, one
    for parameter ``broadcast`` -- so a bucket's broadcast does not queue behind later buckets'
    reduces, and no other ps task contributes zeros to s's traffic;
  - f32 on the wire by default; with ``wire_dtype=torch.bfloat16`` (opt-in) bf16 in both directions: workers pack each gradient bucket f32->bf16 and ``reduce``
    it to the owner; the owner ships back the bf16 COMPUTE copy of weight-decayed buckets (what the
    workers' GEMMs read; the f32 master never leaves the owner) and the small f32 no-decay buckets
    (biases, BN/LayerNorm gamma+beta, which kernels read in f32). Per BERT-base step that is
    ~220 MB up + ~220 MB down per worker instead of 440 + 440 MB in f32;
  - workers launch the ``reduce`` of a bucket the moment backward has produced its last gradient
    (arena readiness callbacks, in bucket order -- the same order on every rank), overlapping the
    rest of backward, exactly like MWMS buckets; the worker step has no host synchronisation and
    is captured in a hipGraph like the MWMS step;
  - the owner zeroes ONLY its own shard's gradient, posts its buckets' reduces, and per bucket:
    stream-waits for that reduce, unpacks it, runs the fused HIP optimizer on the bucket (device LR
    schedule supported: the step advances once per global step), posts its broadcast; so early
    buckets are updated and shipped back while later ones are still being reduced.
  The schedule is identical on every rank (steps and checkpoint steps are known), so no control
  messages are needed; for a checkpoint the owners ``send`` f32 master + slots to the chief.
  The owner loop is host-driven; its run-ahead is bounded (``RUN_AHEAD`` steps, an event ring),
  so a stalled peer shows up as a stalled heartbeat instead of an ever-growing launch queue.
* colocated owners: a shard whose owner is also a worker (``ps_ranks`` ∩ ``worker_ranks``, e.g.
  ``bench.py --strategy ps --force-comm`` at world size 1, where worker 0 owns the only shard) is
  updated inside that worker's own step: its reduce is the worker's reduce, and the unpack ->
  ``step_region`` -> broadcast run in ``apply_gradients`` -- so the whole collective PS path,
  including its hipGraph capture, runs on one GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..runtime.arena import ALIGN, ParamArena
from . import tfk_comm

PUSH, DONE, FETCH, LOAD, PULL = 1, 2, 3, 4, 5
RUN_AHEAD = 2  # owner loop: at most this many global steps enqueued ahead of the device
CAPTURE_OWNER = True  # GPU owners replay their per-step sequence from one hipGraph
OWNER_WARMUP = 2  # eager owner steps before the capture (they size every lazily built table)


def shard_bounds(numel: int, nshards: int, param_spans: list[tuple[int, int]] | None = None) -> list[tuple[int, int]]:
    """Contiguous shards of [0, numel) with near-equal sizes. With param_spans (each parameter's
    [offset, offset+numel) in the arena) every cut falls on a parameter boundary, so no tensor is
    split across two parameter servers: LAMB's per-tensor trust ratio ||w||/||u|| then sees the
    whole tensor on one PS, exactly as in single-process and MWMS training. Without
    spans: ALIGN-aligned cuts."""
    if not param_spans:
        units = (numel + ALIGN - 1) // ALIGN
        out, lo = [], 0
        for s in range(nshards):
            n = units // nshards + (1 if s < units % nshards else 0)
            hi = min(numel, lo + n * ALIGN)
            out.append((lo, hi))
            lo = hi
        return out
    # candidate cut points = parameter ends (sorted, de-duplicated); greedy toward equal byte shares
    ends = sorted({e for _, e in param_spans if 0 < e < numel})
    out, lo = [], 0
    for s in range(nshards):
        if s == nshards - 1:
            out.append((lo, numel))
            break
        target = lo + (numel - lo) / (nshards - s)
        best = None
        for e in ends:
            if e <= lo:
                continue
            if best is None or abs(e - target) < abs(best - target):
                best = e
            if e > target:
                break
        hi = best if best is not None else numel
        out.append((lo, hi))
        lo = hi
    return out


def _param_spans(arena) -> list[tuple[int, int]]:
    return [(p.offset, p.offset + p.numel) for p in arena.params]


def _hdr(cmd: int, step: int = 0, rank: int = 0) -> torch.Tensor:
    return torch.tensor([cmd, step, rank, 0], dtype=torch.int64)


class ParameterServerStrategy:
    """Worker side."""
    name = "ps"

    def __init__(self, arena: ParamArena, ps_ranks: list[int], worker_ranks: list[int], mode: str = "sync",
                 group=None, transport: str = "gloo", bucket_mb: float = 32.0, comm=None, wire_dtype=torch.float32):
        if mode not in ("sync", "async"):
            raise ValueError(f"ps mode must be sync|async, got {mode}")
        if transport not in ("gloo", "rccl"):
            raise ValueError(f"ps transport must be gloo|rccl, got {transport}")
        if transport == "rccl" and mode != "sync":
            raise ValueError("the rccl (collective) transport is synchronous; use transport=gloo for async")
        self.arena, self.ps_ranks, self.worker_ranks, self.mode, self.group = arena, list(ps_ranks), list(worker_ranks), mode, group
        self.transport = transport
        self.comm = comm if comm is not None else tfk_comm.world()
        self.rank = self.comm.rank if self.comm is not None else dist.get_rank()
        self.shards = shard_bounds(arena.numel, len(self.ps_ranks), _param_spans(arena))
        self.plan = None
        if transport == "gloo":
            pin = arena.grad.is_cuda
            self._g = [torch.empty(hi - lo, dtype=torch.float32, pin_memory=pin) for lo, hi in self.shards]
            self._p = [torch.empty(hi - lo, dtype=torch.float32, pin_memory=pin) for lo, hi in self.shards]
        else:
            self.plan = CollectivePlan(arena, self.shards, self.ps_ranks, self.worker_ranks, bucket_mb, self.comm,
                                       wire_dtype)
            arena.on_grad_ready(self._on_ready)
        self.step_count = 0
        self._next = 0
        self._red = []
        # shards this rank owns while also being a worker (colocated owner)
        self.owned = [s for s, owner in enumerate(self.ps_ranks) if owner == self.rank and owner in self.worker_ranks]
        if self.owned and transport != "rccl":
            raise ValueError("a colocated parameter-server shard needs the rccl (collective) transport")

    @property
    def capturable(self) -> bool:
        """The collective worker step (async reduce launches, stream waits on the broadcasts, bf16
        unpack) has no host synchronisation -> hipGraph-capturable; the gloo transport is not."""
        return self.plan is not None and self.comm is not None and self.comm.backend == "rccl"

    def wire_bytes(self) -> int:
        """Bytes one worker moves per step (up + down)."""
        return self.plan.wire_bytes() if self.plan is not None else 2 * 4 * self.arena.numel

    @property
    def num_workers(self) -> int:
        return len(self.worker_ranks)

    def begin_step(self):
        if self.plan is not None:
            self.plan.reset()
            self._next, self._red = 0, []

    def _on_ready(self, p):
        """Backward produced p's gradient: launch every leading complete bucket's reduce."""
        pl = self.plan
        b = pl.bucket_of.get(p.index)
        if b is None:
            return
        pl.pending[b] -= 1
        while self._next < len(pl.buckets) and pl.pending[self._next] <= 0:
            from ..runtime import streams
            # side-stream weight gradients of this bucket: the reduce's comm stream waits on them
            self._red.append(pl.reduce(self._next, self.arena.grad, deps=streams.producers()))
            self._next += 1

    def finish_step(self):
        if self.plan is not None:
            from ..runtime import streams
            deps = streams.producers()
            while self._next < len(self.plan.buckets):
                self._red.append(self.plan.reduce(self._next, self.arena.grad, deps=deps))
                self._next += 1

    def configure_optimizer(self, opt) -> None:
        """The optimizer runs on the ps tasks; the worker-side instance only provides slot names
        and the step counter for checkpoints."""
        self.opt = opt

    def _exchange(self, cmd: int, send: list[torch.Tensor] | None, recv: list[torch.Tensor] | None):
        reqs = []
        for s, ps in enumerate(self.ps_ranks):
            reqs.append(dist.isend(_hdr(cmd, self.step_count, self.rank), ps, group=self.group))
            if send is not None:
                reqs.append(dist.isend(send[s], ps, group=self.group))
        for r in reqs:
            r.wait()
        if recv is not None:
            reqs = [dist.irecv(recv[s], ps, group=self.group) for s, ps in enumerate(self.ps_ranks)]
            for r in reqs:
                r.wait()

    def apply_gradients(self, opt=None) -> None:
        """Push local gradients, pull the updated parameters (replaces optimizer.step())."""
        a = self.arena
        if self.transport == "rccl":
            self.finish_step()  # (no-op when the runner already called it)
            if self.owned:
                self._update_owned(opt if opt is not None else self.opt)
            works = [self.plan.broadcast(i) for i in range(len(self.plan.buckets))]
            for w in self._red + works:
                w.wait()  # stream waits: the next forward is ordered after the pulled parameters
            self._red = []
            self.plan.finish_pull()
            self.step_count += 1
            if opt is not None:
                opt.step_count = self.step_count
            return
        for s, (lo, hi) in enumerate(self.shards):
            self._g[s].copy_(a.grad[lo:hi], non_blocking=True)
        if a.grad.is_cuda:
            torch.cuda.current_stream().synchronize()
        self._exchange(PUSH, self._g, self._p)
        for s, (lo, hi) in enumerate(self.shards):
            a.master[lo:hi].copy_(self._p[s], non_blocking=True)
        a.refresh_compute()
        self.step_count += 1
        if opt is not None:
            opt.step_count = self.step_count

    def _update_owned(self, opt) -> None:
        """Colocated owner: per owned bucket, wait for its reduce, unpack, update (one global step)."""
        plan, k = self.plan, 0
        for s in self.owned:
            for i in plan.buckets_of(s):
                self._red[i].wait()
                plan.unpack(i)
                lo, hi, _ = plan.buckets[i]
                opt.region = (lo, hi)
                opt.step_region(advance=k == 0)
                k += 1
        opt.region = None

    def pull(self) -> None:
        """Initial (or resync) read of every variable from the ps tasks."""
        if self.transport == "rccl":
            self.plan.pull_master()
            return
        self._exchange(PULL, None, self._p)
        for s, (lo, hi) in enumerate(self.shards):
            self.arena.master[lo:hi].copy_(self._p[s])
        self.arena.refresh_compute()

    def fetch_state(self, opt) -> None:
        """Copy master + optimizer slots from the ps tasks into the local arena (chief, before a
        checkpoint save)."""
        names = list(opt.slot_names)
        if self.transport == "rccl":
            dev = self.arena.master.device
            bufs = [torch.empty((1 + len(names)) * (hi - lo), dtype=torch.float32, device=dev) for lo, hi in self.shards]
            for b, ps in zip(bufs, self.ps_ranks):
                self.comm.recv(b, ps)
            if dev.type == "cuda":
                torch.cuda.current_stream().synchronize()
        else:
            bufs = [torch.empty((1 + len(names)) * (hi - lo), dtype=torch.float32) for lo, hi in self.shards]
            self._exchange(FETCH, None, bufs)
        for s, (lo, hi) in enumerate(self.shards):
            n = hi - lo
            self.arena.master[lo:hi].copy_(bufs[s][:n])
            for k, nm in enumerate(names):
                self.arena.slot(nm)[lo:hi].copy_(bufs[s][(k + 1) * n:(k + 2) * n])

    def load_state(self, opt, step: int) -> None:
        """Push master + slots (restored from a checkpoint by the chief) to the ps tasks."""
        names = list(opt.slot_names)
        bufs = []
        for lo, hi in self.shards:
            parts = [self.arena.master[lo:hi].cpu()] + [self.arena.slot(nm)[lo:hi].cpu() for nm in names]
            bufs.append(torch.cat(parts))
        self.step_count = step
        self._exchange(LOAD, bufs, None)

    def shutdown(self) -> None:
        if self.transport == "gloo":
            self._exchange(DONE, None, None)

    def broadcast_parameters(self, src: int = 0):
        self.pull()

    def all_reduce_metrics(self, t: torch.Tensor) -> torch.Tensor:
        return t


class CollectivePlan:
    """Bucket plan + per-shard communicators of the collective PS transport (same on every rank).

    Buckets are parameter-aligned slices of the arena, never crossing a shard boundary or the
    decay/no-decay boundary (so an optimizer region per bucket is valid, LAMB's per-tensor trust
    ratio included), listed in arena order = backward-completion order."""

    def __init__(self, arena: ParamArena, shards, ps_ranks, worker_ranks, bucket_mb: float = 32.0, comm=None,
                 wire_dtype=torch.float32):
        self.arena, self.shards, self.ps_ranks = arena, list(shards), list(ps_ranks)
        self.comm = comm if comm is not None else tfk_comm.world()
        self.me = self.comm.rank
        cap = max(ALIGN, int(bucket_mb * (1 << 20)) // 4)
        cuts = sorted({lo for lo, _ in shards} | {hi for _, hi in shards} | set(arena.decay_region())
                      | set(arena.nodecay_region()))
        params = sorted(arena.params, key=lambda p: p.offset)
        self.buckets: list[tuple[int, int, int]] = []  # (lo, hi, shard)
        self.bucket_of: dict[int, int] = {}
        self._nparams: list[int] = []
        for lo_c, hi_c in zip(cuts, cuts[1:]):
            if hi_c <= lo_c:
                continue
            shard = next(i for i, (a, b) in enumerate(shards) if a <= lo_c < b)
            start, cur = lo_c, []
            for p in params:
                if not (lo_c <= p.offset < hi_c):
                    continue
                cur.append(p)
                end = min(hi_c, p.offset + ((p.numel + ALIGN - 1) // ALIGN) * ALIGN)
                if end - start >= cap:
                    self._add(start, end, shard, cur)
                    start, cur = end, []
            if cur:
                self._add(start, hi_c, shard, cur)
        self.pending = list(self._nparams)
        self.n_decay = arena.n_decay
        # bf16 wire: gradients packed into `wire`, decay-region weights shipped as the bf16 compute copy
        self.wire_dtype = wire_dtype
        self.wire = torch.empty(arena.numel, dtype=wire_dtype, device=arena.grad.device) \
            if wire_dtype != torch.float32 else None
        # two sub-communicators per shard (reduce / broadcast): every rank splits every one, in order
        self.red, self.bc, self.root = [], [], []
        for owner in self.ps_ranks:
            ranks = sorted({owner} | set(worker_ranks))
            self.red.append(self.comm.split(ranks, f"ps{owner}/reduce"))
            self.bc.append(self.comm.split(ranks, f"ps{owner}/bcast"))
            self.root.append(ranks.index(owner))

    def _add(self, lo, hi, shard, params):
        i = len(self.buckets)
        self.buckets.append((lo, hi, shard))
        self._nparams.append(len(params))
        for p in params:
            self.bucket_of[p.index] = i

    def reset(self):
        self.pending = list(self._nparams)

    def buckets_of(self, shard: int) -> list[int]:
        return [i for i, b in enumerate(self.buckets) if b[2] == shard]

    def is_decay(self, i: int) -> bool:
        return self.buckets[i][0] < self.n_decay

    def wire_bytes(self) -> int:
        """Bytes one worker pushes + pulls per step."""
        esz = 4 if self.wire is None else self.wire.element_size()
        up = sum(hi - lo for lo, hi, _ in self.buckets) * esz
        down = sum((hi - lo) * (esz if self.is_decay(i) else 4) for i, (lo, hi, _) in enumerate(self.buckets))
        return up + down

    # ---------------------------------------------------------------- per bucket
    def reduce(self, i: int, grad: torch.Tensor, deps=()):
        """Worker: push bucket i's gradient to its owner (packed to the wire dtype first, on the comm
        stream). deps: the side streams that produced part of the bucket."""
        lo, hi, s = self.buckets[i]
        t = grad[lo:hi]
        pre = None
        if self.wire is not None:
            from ..ops.optim import cast_f32_bf16
            w = self.wire[lo:hi]
            pre = (lambda t=t, w=w: cast_f32_bf16(t, w))
            t = w
        return self.red[s].reduce(t, self.root[s], async_op=True, deps=deps, pre=pre)

    def unpack(self, i: int) -> None:
        """Owner: the reduced bf16 bucket -> f32 gradient (after its reduce completed)."""
        if self.wire is not None:
            from ..ops.optim import cast_bf16_f32
            lo, hi, _ = self.buckets[i]
            cast_bf16_f32(self.wire[lo:hi], self.arena.grad[lo:hi])

    def broadcast(self, i: int):
        """Owner sends / workers receive bucket i's updated weights: the bf16 compute copy for
        weight-decayed buckets (bf16 wire), f32 master for the no-decay buckets."""
        lo, hi, s = self.buckets[i]
        a = self.arena
        t = a.compute[lo:hi] if (self.wire is not None and self.is_decay(i)) else a.master[lo:hi]
        return self.bc[s].broadcast(t, self.root[s], async_op=True)

    def finish_pull(self) -> None:
        """Worker, after every broadcast: refresh the compute copy of what arrived in f32."""
        from ..ops.optim import cast_f32_bf16
        a = self.arena
        if self.wire is None:
            a.refresh_compute()
            return
        lo, hi = a.nodecay_region()
        if hi > lo:
            cast_f32_bf16(a.master[lo:hi], a.compute[lo:hi])

    def pull_master(self) -> None:
        """Initial / resync read of every f32 master shard from its owner (all ranks call)."""
        for s, (lo, hi) in enumerate(self.shards):
            if self.bc[s] is not None:  # another ps task's shard: not a member of its communicator
                self.bc[s].broadcast(self.arena.master[lo:hi], self.root[s])
        self.arena.refresh_compute()


class ParameterServer:
    """ps-task side: owns one shard of the arena (master + slots) and runs the optimizer on it."""

    def __init__(self, arena: ParamArena, opt, shard: int, ps_ranks: list[int], worker_ranks: list[int],
                 mode: str = "sync", group=None):
        self.arena, self.opt, self.mode, self.group = arena, opt, mode, group
        self.worker_ranks = list(worker_ranks)
        self.ps_ranks = list(ps_ranks)
        self.shards = shard_bounds(arena.numel, len(ps_ranks), _param_spans(arena))
        self.lo, self.hi = self.shards[shard]
        opt.region = (self.lo, self.hi)
        if mode == "sync":
            opt.grad_scale = 1.0 / len(self.worker_ranks)
        self.updates = 0

    def _reply(self, dst: int, t: torch.Tensor):
        dist.send(t, dst, group=self.group)

    def _state(self) -> torch.Tensor:
        a, lo, hi = self.arena, self.lo, self.hi
        return torch.cat([a.master[lo:hi]] + [a.slot(nm)[lo:hi] for nm in self.opt.slot_names])

    def _load(self, buf: torch.Tensor, step: int):
        a, lo, hi = self.arena, self.lo, self.hi
        n = hi - lo
        a.master[lo:hi].copy_(buf[:n])
        for k, nm in enumerate(self.opt.slot_names):
            a.slot(nm)[lo:hi].copy_(buf[(k + 1) * n:(k + 2) * n])
        self.opt.step_count = step

    def serve(self, beat=None) -> int:
        """Serve until every worker has sent DONE. Returns the number of optimizer updates.
        ``beat(step)`` is the watchdog heartbeat: called for every command received, so a healthy
        server blocked in recv between worker steps is not mistaken for a hung one -- but a server
        whose workers stop sending is (their gang restart is the recovery)."""
        a, lo, hi = self.arena, self.lo, self.hi
        n = hi - lo
        live = set(self.worker_ranks)
        hdr = torch.empty(4, dtype=torch.int64)
        gbuf = torch.empty(n, dtype=torch.float32)
        pending: list[int] = []  # sync: workers whose push for the current step arrived
        while live:
            src = dist.recv(hdr, None, group=self.group)  # any source
            cmd, step = int(hdr[0]), int(hdr[1])
            if beat is not None:
                beat(step)
            if cmd == DONE:
                live.discard(src)
                continue
            if cmd == PULL:
                self._reply(src, a.master[lo:hi].contiguous())
                continue
            if cmd == FETCH:
                self._reply(src, self._state())
                continue
            if cmd == LOAD:
                buf = torch.empty((1 + len(self.opt.slot_names)) * n, dtype=torch.float32)
                dist.recv(buf, src, group=self.group)
                self._load(buf, step)
                continue
            if cmd != PUSH:
                raise RuntimeError(f"ps: unknown command {cmd} from rank {src}")
            dist.recv(gbuf, src, group=self.group)
            if self.mode == "async":
                a.grad[lo:hi].copy_(gbuf)
                self.opt.step()
                self.updates += 1
                self._reply(src, a.master[lo:hi].contiguous())
                continue
            if not pending:
                a.grad[lo:hi].copy_(gbuf)
            else:
                a.grad[lo:hi].add_(gbuf)
            pending.append(src)
            if len(pending) == len(live):
                self.opt.step()
                self.updates += 1
                out = a.master[lo:hi].contiguous()
                for w in pending:
                    self._reply(w, out)
                pending = []
        return self.updates

    # ------------------------------------------------------------------ rccl transport
    def serve_collective(self, start_step: int, total_steps: int, checkpoint_every: int = 0,
                         chief: int = 0, final_checkpoint: bool = True, bucket_mb: float = 32.0, comm=None,
                         wire_dtype=torch.float32, beat=None) -> int:
        """Mirror of the workers' step schedule over tfk_comm (CollectivePlan): initial broadcast,
        then per step: zero the own shard's gradient, post the own buckets' reduces, and per bucket
        stream-wait -> unpack -> fused optimizer on that bucket -> post its broadcast. The global step
        (host counter or device schedule) advances once per step. Ships f32 master + slots to the
        chief at its checkpoint steps."""
        self.setup_collective(bucket_mb, comm, wire_dtype)
        return self.serve_steps(start_step, total_steps, checkpoint_every, chief, final_checkpoint, beat=beat)

    def setup_collective(self, bucket_mb: float = 32.0, comm=None, wire_dtype=torch.float32) -> None:
        """Create the per-shard sub-communicators (in the same order as the workers'
        ParameterServerStrategy) and serve the initial parameter pull."""
        a = self.arena
        self._comm = comm if comm is not None else tfk_comm.world()
        self._plan = CollectivePlan(a, self.shards, self.ps_ranks, self.worker_ranks, bucket_mb, self._comm, wire_dtype)
        self._plan.pull_master()

    def _owner_step(self, mine) -> None:
        """One global step of this owner's shard, all on streams (hipGraph-capturable): zero the
        own gradient contribution, post the own buckets' reduces, per bucket wait -> unpack ->
        fused optimizer on the bucket -> post its broadcast, then join every broadcast."""
        a, plan, opt = self.arena, self._plan, self.opt
        a.grad[self.lo:self.hi].zero_()  # the owner's own (zero) contribution to its reduces
        if plan.wire is not None:
            plan.wire[self.lo:self.hi].zero_()
        reds = [plan.reduce(i, a.grad) for i in mine]
        bcs = []
        for k, (i, w) in enumerate(zip(mine, reds)):
            w.wait()
            plan.unpack(i)
            lo, hi, _ = plan.buckets[i]
            opt.region = (lo, hi)
            opt.step_region(advance=k == 0)
            bcs.append(plan.broadcast(i))
        for w in bcs:
            w.wait()
        opt.region = (self.lo, self.hi)

    def _capturable(self) -> bool:
        return (self.arena.master.is_cuda and getattr(self._comm, "backend", "") == "rccl"
                and CAPTURE_OWNER and hasattr(self.opt, "enable_device_schedule"))

    def serve_steps(self, start_step: int, end_step: int, checkpoint_every: int = 0, chief: int = 0,
                    final_checkpoint: bool = False, total_steps: int | None = None, beat=None) -> int:
        """Serve global steps start_step+1 .. end_step (after setup_collective). ``beat(step)`` is
        the watchdog heartbeat; the host runs at most RUN_AHEAD steps ahead of the device.

        GPU owners (RCCL transport) capture the step once in a hipGraph after ``OWNER_WARMUP`` eager
        steps and replay it: one host call per global step instead of ~4 per bucket (the learning
        rate, step counter and bias corrections advance on the device, Optimizer.enable_device_schedule).
        The collective sequence is the same captured or eager, so the workers' own graph-or-eager
        decision needs no coordination with the owner; a failed owner capture runs eager
        (``self.capture_fallback`` says why)."""
        a, plan, comm, opt = self.arena, self._plan, self._comm, self.opt
        total = end_step if total_steps is None else total_steps
        me = self.ps_ranks.index(comm.rank)
        mine = plan.buckets_of(me)
        ring = []
        graph = None
        use_graph = self._capturable()
        if use_graph and opt._dev is None:
            opt.step_count = start_step
            opt.enable_device_schedule()
        n_eager = 0
        for step in range(start_step + 1, end_step + 1):
            if len(ring) >= RUN_AHEAD:
                ring.pop(0).synchronize()  # bounded run-ahead: step - RUN_AHEAD has completed
            if beat is not None:
                beat(step)
            if graph is not None:
                graph.replay()
            elif use_graph and n_eager >= OWNER_WARMUP:
                graph = self._capture_owner(mine)
                if graph is None:
                    use_graph = False
                    self._owner_step(mine)
                else:
                    graph.replay()
            else:
                self._owner_step(mine)
                n_eager += 1
            self.updates += 1
            if a.master.is_cuda:
                ev = torch.cuda.Event()
                ev.record()
                ring.append(ev)
            ckpt = (checkpoint_every and step % checkpoint_every == 0 and step < total) or \
                (final_checkpoint and step == total)
            if ckpt:
                comm.send(self._state(), chief)
                if a.master.is_cuda:
                    torch.cuda.current_stream().synchronize()
        self.owner_graph = graph is not None
        if opt._dev is not None:
            opt.sync_step()
        return self.updates

    capture_fallback = ""
    owner_graph = False

    def _capture_owner(self, mine):
        """Capture one owner step (returns None and records why on failure)."""
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._owner_step(mine)
        except Exception as e:  # noqa: BLE001 -- the owner then serves eagerly
            self.capture_fallback = f"{type(e).__name__}: {e}"[:400]
            torch.cuda.synchronize()
            return None
        return g
