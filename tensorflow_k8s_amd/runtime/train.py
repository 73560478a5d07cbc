"""In-pod training entrypoint: ``python -m tensorflow_k8s_amd.runtime.train --model resnet50 ...``.

This is the program a TFJob replica runs (the reference's pods run a TF script that builds a
``TFConfigClusterResolver`` + ``MultiWorkerMirroredStrategy`` / ``ParameterServerStrategy`` from
the operator-injected TF_CONFIG). Per role:

* chief / worker: one process per GPU (HIP_VISIBLE_DEVICES set by the node agent), a tfk_comm RCCL
  world over all workers (MWMS; f32 gradient wire by default, the whole step captured in a hipGraph) or the
  ps tasks (PS strategy: collective RCCL transport, or gloo point-to-point to CPU ps tasks); restore-or-init, train
  ``--steps`` global steps on synthetic data of the model's shape, chief writes TF-bundle
  checkpoints every ``--checkpoint-every`` steps and at the end, JSON-lines metrics on stdout;
* ps: holds one shard of the variables + optimizer slots on the CPU and serves push/pull;
* evaluator: not in the training world; follows the checkpoint directory (runtime/evaluator.py).

Exit codes follow the operator's restart policy (ExitCode): 0 success; 1 permanent user error;
137 OOM (termination message "OOMKilled", permanent) ; 143 peer/rendezvous failure (retryable ->
gang restart, resume from the latest checkpoint). Fault injection for the failure-recovery tests:
TFK_FAULT_AT_STEP=<n> [TFK_FAULT_EXIT=<code>|137=SIGKILL|nan=poison the weights] [TFK_FAULT_RANK=<r>]
[TFK_FAULT_GENERATION=<g>|any, compared with the operator's TFK_RESTART_GENERATION, default 0].
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import time

# hardware queues per process: HIP's default (4); TFK_HW_QUEUES sets it (bench.py, perf_log_r6.md)
if os.environ.get("TFK_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["TFK_HW_QUEUES"]

import torch  # noqa: E402

EXIT_OK, EXIT_USER, EXIT_OOM, EXIT_RETRY = 0, 1, 137, 143


def _log(obj: dict, fh=None):
    line = json.dumps(obj, sort_keys=True)
    print(line, flush=True)
    if fh is not None:
        fh.write(line + "\n")
        fh.flush()


def _termination_message(msg: str):
    path = os.environ.get("TFK_TERMINATION_LOG")
    if path:
        try:
            with open(path, "w") as f:
                f.write(msg)
        except OSError:
            pass


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model", default="lenet")
    ap.add_argument("--batch", type=int, default=64, help="per-worker batch")
    ap.add_argument("--steps", type=int, default=100, help="total global steps")
    ap.add_argument("--optimizer", default="sgd", choices=["sgd", "adamw", "lamb"])
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight-decay", type=float, default=0.0)
    ap.add_argument("--warmup-steps", type=int, default=0)
    ap.add_argument("--lr-schedule", default="constant", choices=["constant", "cosine", "poly"])
    ap.add_argument("--strategy", default="auto", choices=["auto", "mwms", "ps"])
    ap.add_argument("--ps-mode", default="sync", choices=["sync", "async"])
    ap.add_argument("--ps-transport", default="gloo", choices=["gloo", "rccl"],
                    help="gloo: ps tasks on CPU (sync/async); rccl: ps tasks own a GPU, RCCL reduce/broadcast (sync)")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--comm-dtype", default="f32", choices=["f32", "bf16"],
                    help="gradient wire dtype (MWMS all-reduce, collective PS push/pull); f32 default = exact f32 "
                         "aggregation, bf16 = half the xGMI bytes (opt-in, like TF's CommunicationOptions)")
    ap.add_argument("--device", default="auto", choices=["auto", "cpu", "cuda"])
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a hipGraph (default: on for GPU workers at any world size, unless the "
                         "model has host-side per-step state)")
    ap.add_argument("--checkpoint-dir", default="")
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--keep", type=int, default=5)
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--metrics-file", default="")
    ap.add_argument("--data-batches", type=int, default=4, help="distinct synthetic batches per worker")
    ap.add_argument("--image-size", type=int, default=0, help="override input resolution (ResNet)")
    ap.add_argument("--num-classes", type=int, default=0)
    ap.add_argument("--seq-len", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--step-sleep", type=float, default=0.0, help="seconds to pause after each step (paces demo/test jobs)")
    ap.add_argument("--rendezvous-timeout", type=float, default=300.0)
    ap.add_argument("--watchdog-timeout", type=float, default=-1.0,
                    help="abort the communicators and exit 143 (retryable) when no step completes for this many "
                         "seconds or RCCL reports an async error (default: 300 s at world size > 1; 0 = off)")
    ap.add_argument("--trace-file", default="", help="Chrome-trace step timeline (+ roctx ranges); {rank} expands")
    # evaluator
    ap.add_argument("--eval-batches", type=int, default=4)
    ap.add_argument("--eval-timeout", type=float, default=600.0)
    args = ap.parse_args(argv)
    for k in ("checkpoint_dir", "metrics_file", "trace_file"):
        setattr(args, k, volume_path(getattr(args, k)))
    return args


def volume_path(p: str) -> str:
    """A path under a volumeMount's mountPath -> the host directory behind it, when the kubelet ran
    this container without a mount namespace (TFK_VOLUME_MAP="<mountPath>=<hostDir>;..."; the kubelet
    already rewrote the paths in args/env, this covers ones from config files or code)."""
    vm = os.environ.get("TFK_VOLUME_MAP", "")
    if not p or not vm:
        return p
    best = None
    for ent in vm.split(";"):
        dst, _, src = ent.partition("=")
        if dst and (p == dst or p.startswith(dst.rstrip("/") + "/")) and (best is None or len(dst) > len(best[0])):
            best = (dst, src)
    return best[1] + p[len(best[0]):] if best else p


def model_kwargs(args) -> dict:
    kw = {}
    if args.num_classes:
        kw["num_classes"] = args.num_classes
    if args.model.startswith("lenet") and args.image_size:
        kw["image_size"] = args.image_size
    return kw


def data_kwargs(args) -> dict:
    kw = {}
    if args.image_size:
        kw["image_size"] = args.image_size
    if args.seq_len:
        kw["seq_len"] = args.seq_len
    return kw


def make_optimizer(args, arena):
    from .optimizer import LAMB, SGD, AdamW, LRSchedule
    lr = LRSchedule(args.lr, warmup=args.warmup_steps, total=args.steps, kind=args.lr_schedule)
    if args.optimizer == "sgd":
        return SGD(arena, lr, momentum=args.momentum, weight_decay=args.weight_decay)
    if args.optimizer == "adamw":
        return AdamW(arena, lr, weight_decay=args.weight_decay)
    return LAMB(arena, lr, weight_decay=args.weight_decay)


def pick_device(args, info) -> torch.device:
    if (info.is_ps and args.ps_transport == "gloo") or args.device == "cpu":
        return torch.device("cpu")
    want_cuda = args.device == "cuda" or (args.device == "auto" and torch.cuda.is_available())
    if not want_cuda:
        return torch.device("cpu")
    if not torch.cuda.is_available():
        raise SystemExit("--device cuda but no GPU is visible")
    # torchrun: LOCAL_RANK; a TFJob pod: TFK_LOCAL_DEVICE (its GPU in the visible list -- all of the
    # gang's GPUs under the gang-visible-gpus opt-in, else just its own)
    local = int(os.environ.get("LOCAL_RANK", "0")) if info.source == "torchrun" else \
        int(os.environ.get("TFK_LOCAL_DEVICE", "0"))
    torch.cuda.set_device(local)
    return torch.device("cuda", local)


def maybe_fault(step: int, rank: int, arena=None):
    at = os.environ.get("TFK_FAULT_AT_STEP")
    if not at or int(at) != step:
        return
    if int(os.environ.get("TFK_FAULT_RANK", "0")) != rank:
        return
    gen = os.environ.get("TFK_FAULT_GENERATION", "0")
    if gen != "any" and gen != os.environ.get("TFK_RESTART_GENERATION", "0"):
        return
    if os.environ.get("TFK_FAULT_EXIT") == "nan":
        # silent corruption instead of a crash: the next steps' loss is NaN (the numerics guard's case)
        _log({"event": "fault_injected", "step": step, "rank": rank, "exit": "nan"})
        if arena is not None:
            arena.master.fill_(float("nan"))
            arena.compute.fill_(float("nan"))
        return
    code = int(os.environ.get("TFK_FAULT_EXIT", "1"))
    _log({"event": "fault_injected", "step": step, "rank": rank, "exit": code})
    sys.stdout.flush()
    if code == 137:
        os.kill(os.getpid(), signal.SIGKILL)
    os._exit(code)


def _beats(watchdog):
    """Heartbeat callback of a serving loop: the liveness file (runtime/health.py) + the watchdog."""
    from . import health

    def beat(*a, **k):
        health.beat()
        if watchdog is not None:
            watchdog.beat(*a, **k)
    return beat


def run_ps(args, info, dev, world_comm, watchdog=None) -> int:
    from ..models import build_model
    from ..parallel import tfk_comm
    from ..parallel.ps import ParameterServer
    from .checkpoint import CheckpointManager
    model = build_model(args.model, **model_kwargs(args)).to(dev, seed=args.seed)
    opt = make_optimizer(args, model.arena)
    start = 0
    if args.checkpoint_dir:
        step = CheckpointManager(args.checkpoint_dir, args.keep).restore(model.arena, opt)
        if step is not None:
            start = step
            _log({"event": "restored", "role": "ps", "step": step, "index": info.task_index})
    shard = info.ps_ranks.index(info.rank)
    server = ParameterServer(model.arena, opt, shard, info.ps_ranks, info.worker_ranks, args.ps_mode)
    _log({"event": "ps_ready", "index": info.task_index, "shard": [server.lo, server.hi],
          "transport": args.ps_transport, "device": str(dev)})
    if args.ps_transport == "rccl":
        n = server.serve_collective(start, args.steps, args.checkpoint_every if args.checkpoint_dir else 0,
                                    chief=0, final_checkpoint=bool(args.checkpoint_dir), bucket_mb=args.bucket_mb,
                                    comm=world_comm, wire_dtype=_wire(args),
                                    beat=_beats(watchdog))
    else:
        n = server.serve(beat=_beats(watchdog))
    _log({"event": "done", "role": "ps", "index": info.task_index, "updates": n})
    if watchdog is not None:
        watchdog.exit_code = 0  # the job's part is done: a hung teardown is not a failure
    tfk_comm.shutdown()
    return EXIT_OK


def _wire(args):
    return torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32


def run_worker(args, info, dev, world_comm, watchdog=None) -> int:
    from ..models import build_model, synthetic_batch
    from ..parallel import tfk_comm
    from .checkpoint import CheckpointManager
    from .trainer import StepRunner

    use_ps = args.strategy == "ps" or (args.strategy == "auto" and info.ps_ranks)
    model = build_model(args.model, **model_kwargs(args)).to(dev, seed=args.seed)
    if hasattr(model, "rng_stream"):
        model.rng_stream = info.rank  # each replica draws its own dropout masks
    opt = make_optimizer(args, model.arena)
    if use_ps:
        from ..parallel.ps import ParameterServerStrategy
        if not info.ps_ranks:
            raise SystemExit("--strategy ps needs ps tasks in TF_CONFIG")
        strat = ParameterServerStrategy(model.arena, info.ps_ranks, info.worker_ranks, args.ps_mode,
                                        transport=args.ps_transport, bucket_mb=args.bucket_mb, comm=world_comm,
                                        wire_dtype=_wire(args))
        strat.configure_optimizer(opt)
    else:
        from ..parallel.mwms import MultiWorkerMirroredStrategy
        strat = MultiWorkerMirroredStrategy(model.arena, comm=world_comm, bucket_mb=args.bucket_mb,
                                            comm_dtype=args.comm_dtype)
        strat.configure_optimizer(opt)
    nworkers = max(1, len(info.worker_ranks))
    wrank = info.worker_ranks.index(info.rank) if info.rank in info.worker_ranks else 0

    ckpt = CheckpointManager(args.checkpoint_dir, args.keep) if args.checkpoint_dir else None
    _ACTIVE["ckpt"] = ckpt
    start = 0
    if ckpt is not None:
        s = ckpt.restore(model.arena, opt)
        if s is not None:
            start = s
            _log({"event": "restored", "step": s, "rank": info.rank, "path": ckpt.latest()})
    strat.broadcast_parameters()  # MWMS: chief's weights everywhere; PS: pull from the ps tasks
    if use_ps:
        strat.step_count = start

    batches = [synthetic_batch(model, args.batch, dev, seed=args.seed * 7919 + wrank * 1009 + i, **data_kwargs(args))
               for i in range(max(1, args.data_batches))]
    static = tuple(t.clone() for t in batches[0])
    from .trainer import graph_hazards
    use_graph = dev.type == "cuda" and (not graph_hazards(model) if args.graph < 0 else bool(args.graph))
    agree, probe = None, "off"
    if world_comm is not None and world_comm.backend == "rccl":
        # graph-or-eager decided unanimously by the workers (runtime/guard.py): probe capture of
        # fork -> all_reduce -> join (MWMS), then a vote on the real step's capture
        from .guard import Agreement, capture_probe
        agree = Agreement(world_comm.store, info.rank, info.worker_ranks, timeout_s=args.rendezvous_timeout)
        if use_graph and not use_ps:
            if watchdog is not None:
                watchdog.beat(phase="capture probe")
            use_graph, probe = capture_probe(world_comm, agree, info.rank)
    runner = StepRunner(model, opt, strat, static, use_graph=use_graph, agree=agree, rank=info.rank)
    metrics_fh = open(args.metrics_file, "a") if (args.metrics_file and info.is_chief) else None
    gb = args.batch * nworkers
    _log({"event": "start", "rank": info.rank, "world": info.world_size, "workers": nworkers, "model": model.name,
          "params": model.arena.num_parameters(), "device": str(dev), "strategy": strat.name, "start_step": start,
          "wire_mb_per_step": round(strat.wire_bytes() / 2**20, 3) if hasattr(strat, "wire_bytes") else 0.0,
          "hipgraph": runner.use_graph, "capture_probe": probe,
          "global_batch": gb, "restart_generation": int(os.environ.get("TFK_RESTART_GENERATION", "0"))})
    from ..utils.tracing import NULL_TRACER, Tracer
    tracer = Tracer(rank=info.rank, device_events=dev.type == "cuda") if args.trace_file else NULL_TRACER
    if watchdog is not None:
        watchdog.beat(start, phase="train")
    t_last, n_last = time.perf_counter(), 0
    fell_back = False
    step = start
    from . import health
    while step < args.steps:
        health.beat()
        with tracer.span("step", cat="train", step=step):
            runner.set_batch(*batches[step % len(batches)])
            runner.step()
        step += 1
        n_last += 1
        if watchdog is not None:
            if dev.type == "cuda":
                # follow the device: a replayed graph returns at once, so the heartbeat is the
                # completion of an event recorded after the step (runtime/watchdog.py)
                ev = torch.cuda.Event()
                ev.record()
                watchdog.beat_device(step, ev)
            else:
                watchdog.beat(step)
        if runner.fallback and not fell_back:
            fell_back = True
            _log({"event": "graph_fallback", "rank": info.rank, "step": step, "reason": runner.fallback[:500]})
        # (same on every rank: the metrics reduction below is a collective)
        ckpt_due = bool(ckpt is not None and args.checkpoint_every and step % args.checkpoint_every == 0
                        and step < args.steps)
        if step % max(1, args.log_every) == 0 or step == args.steps or ckpt_due:
            # [loss, accuracy, embedding-guard events]: summed over the workers so every rank sees the
            # same verdict and a corrupt step fails the job before anything is logged or checkpointed
            m = torch.tensor([runner.last_loss() or 0.0, runner.last_accuracy() or 0.0, float(_emb_guard(dev))],
                             dtype=torch.float32, device=dev if strat.name == "mwms" else "cpu")
            strat.all_reduce_metrics(m)
            if strat.name == "mwms":
                m /= nworkers
            if dev.type == "cuda":
                torch.cuda.synchronize()
            _check_numerics(step, float(m[0]), float(m[2]))
            now = time.perf_counter()
            if info.is_chief:
                _log({"event": "train", "step": step, "loss": round(float(m[0]), 6), "accuracy": round(float(m[1]), 6),
                      "examples_per_sec": round(gb * n_last / max(now - t_last, 1e-9), 2),
                      "lr": opt.lr(step - 1)}, metrics_fh)
            t_last, n_last = now, 0
        if ckpt_due and info.is_chief:
            with tracer.span("checkpoint", cat="io", step=step):
                if use_ps:
                    strat.fetch_state(opt)
                    opt.step_count = step  # the ps tasks ran the updates (a captured step keeps no host count)
                path = ckpt.save(model.arena, opt, step)
            _log({"event": "checkpoint", "step": step, "path": path}, metrics_fh)
        maybe_fault(step, info.rank, model.arena)
        if args.step_sleep > 0:
            time.sleep(args.step_sleep)
    if args.trace_file:
        _log({"event": "trace", "path": tracer.dump(args.trace_file.format(rank=info.rank))})
    if ckpt is not None and info.is_chief:
        if use_ps:
            strat.fetch_state(opt)
            opt.step_count = step
        path = ckpt.save(model.arena, opt, step, blocking=True)
        _log({"event": "checkpoint", "step": step, "path": path, "final": True}, metrics_fh)
        with open(os.path.join(args.checkpoint_dir, "DONE"), "w") as f:
            f.write(str(step))
    if use_ps:
        strat.shutdown()
    if world_comm is not None and not use_ps:
        world_comm.barrier()
    if watchdog is not None:
        # the result is out: the communicator teardown below must not be mistaken for an RCCL error
        # (a destroyed communicator reports "aborted") or a hang turned into a retryable failure
        watchdog.exit_code = 0
        watchdog.stop()
    tfk_comm.shutdown()
    if info.is_chief:
        _log({"event": "done", "step": step, "loss": runner.last_loss()}, metrics_fh)
    return EXIT_OK


class NumericsError(RuntimeError):
    """A training step produced a non-finite loss or out-of-range embedding ids: permanent (a restart
    from the last checkpoint would replay the same data and weights)."""


def _emb_guard(dev) -> int:
    """Out-of-range events the bucketed embedding backward skipped since the last read (GPU only)."""
    if dev.type != "cuda":
        return 0
    from ..ops._lib import lib
    return int(lib().emb_guard_count())


def _check_numerics(step: int, loss: float, emb_guard: float) -> None:
    import math
    if not math.isfinite(loss):
        raise NumericsError(f"NonFiniteLoss: loss {loss} at step {step}")
    if emb_guard > 0:
        raise NumericsError(f"EmbeddingGuard: {emb_guard:g} out-of-range embedding events by step {step}")


def _guard_error():
    from .guard import CommSelfTestError
    return CommSelfTestError


# the replica's in-flight state a graceful stop must not lose (SIGTERM handler below)
_ACTIVE: dict = {}
TERM_FLUSH_S = float(os.environ.get("TFK_TERM_FLUSH_S", "10"))


def _on_sigterm(signum, frame):
    """Graceful stop (gang restart, resize, job deletion: the kubelet's SIGTERM before its SIGKILL
    deadline): let an asynchronous checkpoint write that is in flight finish -- the newest
    checkpoint is what the next generation resumes from -- then exit 143 (retryable)."""
    mgr = _ACTIVE.get("ckpt")
    t = getattr(mgr, "_thread", None)
    flushed = False
    if t is not None and t.is_alive():
        t.join(timeout=TERM_FLUSH_S)
        flushed = not t.is_alive()
    _log({"event": "terminated", "signal": int(signum), "checkpoint_flushed": flushed})
    sys.stdout.flush()
    os._exit(EXIT_RETRY)


def main(argv=None) -> int:
    args = parse_args(argv)
    signal.signal(signal.SIGTERM, _on_sigterm)
    from . import health
    health.beat(force=True)  # alive; later beats: setup phases and every step
    from ..parallel import cluster
    from .checkpoint import CheckpointWriteError
    info = cluster.resolve()
    if info.is_evaluator:
        from .evaluator import run_evaluator
        return run_evaluator(args)
    try:
        dev = pick_device(args, info)
        if dev.type == "cpu" and info.world_size > 1 and "OMP_NUM_THREADS" not in os.environ:
            # co-located CPU replicas: split the cores instead of oversubscribing them
            torch.set_num_threads(max(1, (os.cpu_count() or 1) // info.world_size))
        world_comm = None
        watchdog = None
        wd_s = args.watchdog_timeout if args.watchdog_timeout >= 0 else (300.0 if info.world_size > 1 else 0.0)
        if wd_s > 0:
            # failure detection: heartbeat + ncclCommGetAsyncError polling from the
            # first collective on; a hung/failed peer aborts the communicators and exits 143
            from .watchdog import StepWatchdog
            watchdog = StepWatchdog(wd_s, name=f"rank{info.rank}", comm_checks=True).start()
            watchdog.beat(phase="rendezvous")
        if info.world_size > 1:
            use_ps = args.strategy == "ps" or (args.strategy == "auto" and info.ps_ranks)
            backend = "rccl" if (dev.type == "cuda" and (not use_ps or args.ps_transport == "rccl")) else "gloo"
            world_comm = cluster.init_comm(info, dev, backend, timeout_s=args.rendezvous_timeout,
                                           retries=int(os.environ.get("TFK_RENDEZVOUS_RETRIES", "5")))
            if watchdog is not None:
                watchdog.beat(phase="comm self-test")
            from .guard import comm_self_test
            _log({"event": "comm_self_test", "rank": info.rank, **comm_self_test(world_comm)})
            if watchdog is not None:
                watchdog.beat(phase="setup")
            health.beat()
        try:
            if info.is_ps:
                return run_ps(args, info, dev, world_comm, watchdog)
            return run_worker(args, info, dev, world_comm, watchdog)
        finally:
            if watchdog is not None:
                watchdog.stop()
    except torch.cuda.OutOfMemoryError as e:
        _termination_message("OOMKilled")
        _log({"event": "error", "kind": "oom", "message": str(e)[:500]})
        return EXIT_OOM
    except CheckpointWriteError as e:
        # permanent (a restart would hit the same full disk); the previous checkpoint is intact
        _termination_message(f"CheckpointWriteFailed: {e}"[:2000])
        _log({"event": "error", "kind": "checkpoint", "message": str(e)[:500]})
        return EXIT_USER
    except NumericsError as e:
        _termination_message(str(e))
        _log({"event": "error", "kind": "numerics", "message": str(e)[:500]})
        return EXIT_USER
    except (cluster.RendezvousError, _guard_error()) as e:
        _termination_message(str(e))
        _log({"event": "error", "kind": "rendezvous", "message": str(e)[:500]})
        return EXIT_RETRY
    except (RuntimeError, ConnectionError, OSError) as e:
        msg = str(e)
        import torch.distributed as dist
        peer = isinstance(e, getattr(dist, "DistBackendError", ())) or any(
            k in msg for k in ("Connection reset", "Connection closed", "timed out", "Timeout", "NCCL", "RCCL",
                               "gloo", "Broken pipe", "peer"))
        _termination_message(msg[:2000])
        _log({"event": "error", "kind": "peer" if peer else "runtime", "message": msg[:500]})
        return EXIT_RETRY if peer else EXIT_USER


if __name__ == "__main__":
    code = main()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)
