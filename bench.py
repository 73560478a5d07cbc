#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole job) of ResNet-50 bf16 MultiWorkerMirroredStrategy
training on N MI355X GPUs of one node (BASELINE.json metric/config).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

One process per GPU (RANK/LOCAL_RANK/WORLD_SIZE from the launcher), RCCL over xGMI for the
bucketed gradient all-reduce, hand-written gfx950 HIP kernels for conv/BN/pool/loss/SGD.
Synthetic ImageNet-shaped data (on-device, fixed batch) and random-init weights. The timed
region is exactly K full training steps (forward, backward, all-reduce, fused SGD update),
bracketed by barrier + device synchronize; rank 0 prints one JSON line with the MAX over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# Hardware queues per process (read by the HIP runtime when it initializes): HIP's default 4. 8 was
# 0.5 % faster without collectives but 6.4 ms/step slower with the RCCL comm stream in the captured
# step (profiles/perf_log_r6.md); TFK_HW_QUEUES sets it for experiments.
if os.environ.get("TFK_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["TFK_HW_QUEUES"]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: 256 ResNet, 64 BERT, 32 Transformer)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--strategy", default="mwms", choices=["mwms", "ps"],
                    help="mwms: all-reduce data parallelism; ps: ParameterServerStrategy (the last --ps ranks serve)")
    ap.add_argument("--ps", type=int, default=2, help="--strategy ps: number of parameter-server ranks")
    ap.add_argument("--ps-transport", default="rccl", choices=["rccl", "gloo"],
                    help="rccl: ps ranks own a GPU (bucketed bf16 reduce/broadcast); gloo: ps ranks on the CPU")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--comm-dtype", default="f32", choices=["bf16", "f32"],
                    help="gradient wire dtype (f32 default: exact f32 aggregation like TF's; bf16: half the xGMI "
                         "bytes, opt-in like TF's CommunicationOptions; f32 master update either way)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the step in a hipGraph (default: on, at every world size, unless the model has host-side per-step state)")
    ap.add_argument("--rccl-algo", default="", help="RCCL algorithm (Ring|Tree|...), see parallel/comm.py")
    ap.add_argument("--rccl-proto", default="", help="RCCL protocol (Simple|LL|LL128)")
    ap.add_argument("--rccl-channels", type=int, default=0, help="minimum RCCL channels (concurrent rings)")
    ap.add_argument("--watchdog-timeout", type=float, default=-1.0,
                    help="abort the communicators and exit 143 after this many seconds without progress, or at "
                         "once on an RCCL async error (default: 300 s when the step has collectives, else off)")
    ap.add_argument("--force-comm", action="store_true",
                    help="1 GPU: still run the RCCL gradient all-reduce (world-size-1 tfk_comm communicator)")
    ap.add_argument("--fp8", type=int, default=0, help="transformer models: MX-fp8 linear GEMMs (fwd, dgrad, wgrad)")
    ap.add_argument("--mx-wgrad", type=int, default=-1, help=argparse.SUPPRESS)  # A/B: fp8 weight gradients
    ap.add_argument("--via-operator", action="store_true",
                    help="measure through a TFJob: tfk-cluster gang-schedules one pod per GPU (TF_CONFIG rendezvous)")
    ap.add_argument("--tfjob-worker", action="store_true", help=argparse.SUPPRESS)  # a pod of --via-operator
    # CPU rehearsal of the multi-rank code path (gloo, fp32 CPU executor; tests only -- not a measurement)
    ap.add_argument("--cpu-rehearsal", action="store_true", help=argparse.SUPPRESS)
    # tests: report the L2 norm / sum of the master-weight change over the run (graph vs eager parity)
    ap.add_argument("--report-update", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.via_operator:
        return run_via_operator(args)
    if not args.batch:
        args.batch = 256 if args.model.startswith("resnet") else (64 if args.model.startswith("bert") else 32)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    info = None
    if args.tfjob_worker:
        # one pod per GPU (HIP_VISIBLE_DEVICES pinned by the kubelet): the world comes from TF_CONFIG
        from tensorflow_k8s_amd.parallel import cluster
        info = cluster.resolve()
        # TFK_LOCAL_DEVICE: this pod's GPU within the visible list (gang-visible pods see all the
        # gang's GPUs, so RCCL can reach its peers over xGMI P2P/IPC)
        world, rank, local = info.world_size, info.rank, int(os.environ.get("TFK_LOCAL_DEVICE", "0"))
    if args.gpus > 1 and world == 1:
        sys.exit("for --gpus > 1 launch with: python -m torch.distributed.run --nproc-per-node N "
                 "--master-addr 127.0.0.1 bench.py --gpus N")
    # roles: parameter servers are the last ranks (TF_CONFIG order: chief, workers, ps)
    if info is not None:
        ps_ranks, worker_ranks = list(info.ps_ranks), list(info.worker_ranks)
    elif args.strategy == "ps" and args.force_comm and world == 1:
        # colocated: worker 0 also owns the only shard -- the collective PS path on one GPU
        ps_ranks, worker_ranks = [0], [0]
    else:
        nps = args.ps if args.strategy == "ps" else 0
        ps_ranks, worker_ranks = list(range(world - nps, world)), list(range(world - nps))
    use_ps = args.strategy == "ps" or bool(ps_ranks)
    if use_ps and (not ps_ranks or not worker_ranks):
        sys.exit(f"--strategy ps needs at least one worker and one ps rank (world {world}, --ps {args.ps})")
    is_ps = rank in ps_ranks and rank not in worker_ranks
    ps_on_cpu = (use_ps and args.ps_transport == "gloo") or args.cpu_rehearsal
    if (is_ps and ps_on_cpu) or args.cpu_rehearsal:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)

    from tensorflow_k8s_amd.parallel import comm, tfk_comm
    rccl_cfg = comm.configure_rccl(args.rccl_algo or None, args.rccl_proto or None, args.rccl_channels)
    if (world > 1 or args.force_comm) and not ps_on_cpu:
        comm.enable_transport_log()
    # the world communicator is the runtime's own RCCL binding (parallel/tfk_comm.py): no
    # torch.distributed process group, collectives enqueued on a comm stream the step graph captures
    # (gloo only when the parameter servers live on the CPU)
    world_comm = None
    cdev = torch.device("cpu") if ps_on_cpu else dev
    if world > 1:
        if info is not None:
            from tensorflow_k8s_amd.parallel import cluster
            world_comm = cluster.init_comm(info, cdev, "gloo" if ps_on_cpu else "rccl", timeout_s=300)
        else:
            world_comm = tfk_comm.init(tfk_comm.env_store(rank, world), rank, world, cdev)
    elif args.force_comm:
        import torch.distributed as dist
        world_comm = tfk_comm.init(dist.HashStore(), 0, 1, dev)
    # failure detection from here on: heartbeat + ncclCommGetAsyncError polling; a hung or failed
    # collective aborts every communicator and exits 143 (retryable) instead of wedging the node
    wd = None
    wd_s = args.watchdog_timeout if args.watchdog_timeout >= 0 else (300.0 if world_comm is not None else 0.0)
    if wd_s > 0:
        from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog
        wd = StepWatchdog(wd_s, name=f"bench-rank{rank}", comm_checks=True).start()
        wd.beat(phase="comm self-test")
    guards = {}
    if world_comm is not None:
        # the interconnect is checked before any model work: exact all-reduce + broadcast results
        from tensorflow_k8s_amd.runtime.guard import comm_self_test
        guards["comm_self_test"] = comm_self_test(world_comm)
    # barrier / timing group: the workers (parameter servers serve on their own schedule)
    wcomm = world_comm.split(worker_ranks, "workers") if (use_ps and world_comm is not None) else world_comm
    if wd is not None:
        wd.beat(phase="setup")

    from tensorflow_k8s_amd.models import build_model, synthetic_batch
    from tensorflow_k8s_amd.runtime.optimizer import LAMB, SGD, AdamW
    from tensorflow_k8s_amd.runtime.trainer import StepRunner

    is_cnn = args.model.startswith("resnet")
    nworkers = len(worker_ranks)
    if args.mx_wgrad >= 0:
        from tensorflow_k8s_amd.ops import fp8 as _F8
        _F8.MX_WGRAD = bool(args.mx_wgrad)
    model = build_model(args.model, **({"fp8": True} if args.fp8 else {})).to(dev)
    if hasattr(model, "rng_stream"):
        model.rng_stream = rank  # each replica draws its own dropout masks
    if is_cnn:
        opt = SGD(model.arena, lr=0.1 * args.batch * nworkers / 256, momentum=0.9, weight_decay=5e-5)
        opt_name = "SGD momentum 0.9 (fused HIP)"
    elif args.model.startswith("bert"):
        opt = LAMB(model.arena, lr=1e-4, weight_decay=0.01)
        opt_name = "LAMB (fused HIP)"
    else:
        opt = AdamW(model.arena, lr=1e-4, b2=0.98, eps=1e-9, weight_decay=0.0)
        opt_name = "Adam (fused HIP)"
    wire = torch.bfloat16 if args.comm_dtype == "bf16" else torch.float32

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    if is_ps:
        # parameter-server rank: holds one shard (f32 master + slots), serves every worker step
        from tensorflow_k8s_amd.parallel.ps import ParameterServer
        server = ParameterServer(model.arena, opt, ps_ranks.index(rank), ps_ranks, worker_ranks, "sync")
        if wd is not None:
            wd.beat(phase="serve")
        if args.ps_transport == "gloo":
            server.serve(beat=wd.beat if wd is not None else None)
        else:
            server.setup_collective(args.bucket_mb, world_comm, wire)
            server.serve_steps(0, args.warmup + args.steps, beat=wd.beat if wd is not None else None)
            sync()
        _gather_times(world_comm, cdev, world, 0.0)  # (the workers' clock defines the result)
        if wd is not None:
            wd.exit_code = 0
        tfk_comm.shutdown()
        if wd is not None:
            wd.stop()
        return 0

    if use_ps:
        from tensorflow_k8s_amd.parallel.ps import ParameterServerStrategy
        strat = ParameterServerStrategy(model.arena, ps_ranks, worker_ranks, "sync", transport=args.ps_transport,
                                        bucket_mb=args.bucket_mb, comm=world_comm, wire_dtype=wire)
        strat_name = f"ParameterServerStrategy ps={len(ps_ranks)} worker={nworkers} ({args.ps_transport} transport)"
    else:
        from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
        strat = MultiWorkerMirroredStrategy(model.arena, comm=world_comm, bucket_mb=args.bucket_mb,
                                            comm_dtype=args.comm_dtype, force=args.force_comm)
        strat_name = "MultiWorkerMirroredStrategy (tfk_comm RCCL all-reduce)"
    strat.configure_optimizer(opt)
    strat.broadcast_parameters()
    master0 = model.arena.master.clone() if args.report_update else None
    batch = synthetic_batch(model, args.batch, dev, seed=1000 + rank)
    # the whole step (fwd, bwd, RCCL bucket collectives, optimizer) replays from one hipGraph at every
    # world size; only a model with host-side per-step state (graph_hazards) runs eager
    from tensorflow_k8s_amd.runtime.trainer import graph_hazards
    use_graph = (not graph_hazards(model)) if args.graph < 0 else bool(args.graph)
    agree = None
    if wcomm is not None:
        # graph-or-eager is decided unanimously by the ranks that share the step's collectives: a
        # probe capture of fork -> all_reduce -> join first, then a vote on the real step's capture
        from tensorflow_k8s_amd.runtime.guard import Agreement, capture_probe
        agree = Agreement(wcomm.store, rank, worker_ranks)
        if use_graph:
            if wd is not None:
                wd.beat(phase="capture probe")
            ok, why = capture_probe(wcomm, agree, rank)
            guards["capture_probe"] = why
            use_graph = ok
        else:
            guards["capture_probe"] = "off"
    runner = StepRunner(model, opt, strat, batch, use_graph=use_graph, agree=agree, rank=rank)
    beat = (lambda i, ph="train": wd.beat(i, ph)) if wd is not None else (lambda i, ph="train": None)

    def barrier():
        sync()
        if wcomm is not None:
            wcomm.barrier()
        sync()

    for i in range(args.warmup):
        runner.step()
        beat(i, "warmup")
    barrier()
    # per-step device timestamps (no host sync inside the timed loop) for the median / p90
    gpu = dev.type == "cuda"
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if gpu else []
    t0 = time.perf_counter()
    if gpu:
        evs[0].record()
    for i in range(args.steps):
        runner.step()
        if gpu:
            evs[i + 1].record()
            if wd is not None:
                wd.beat_device(args.warmup + i, evs[i + 1], "train")  # device completion, not enqueue
                continue
        beat(args.warmup + i)
    barrier()
    dt = time.perf_counter() - t0
    mine_ms = dt / args.steps * 1000.0
    if use_ps and args.ps_transport == "gloo":
        strat.shutdown()  # DONE to the CPU parameter servers (their serve() loop ends)
    dt, per_rank = _gather_times(world_comm, cdev, world, mine_ms, worker_ranks)
    ms = dt
    step_ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)) if gpu else [ms] * args.steps
    dist_ms = {"median": round(step_ms[len(step_ms) // 2], 3),
               "p90": round(step_ms[min(len(step_ms) - 1, int(0.9 * len(step_ms)))], 3),
               "min": round(step_ms[0], 3), "max": round(step_ms[-1], 3)}
    gb = args.batch * nworkers
    value = gb / (ms / 1000.0)
    comm_cfg = {"comm_dtype": args.comm_dtype, "bucket_mb": args.bucket_mb}
    if use_ps:
        comm_cfg.update({"ps_ranks": ps_ranks, "worker_ranks": worker_ranks, "transport": args.ps_transport,
                         "buckets": len(strat.plan.buckets) if strat.plan is not None else 0,
                         "wire_mb_per_step": round(strat.wire_bytes() / 2**20, 1)})
        enabled = True
    else:
        comm_cfg.update({"buckets": len(strat.buckets),
                         "wire_mb_per_step": round(strat.wire_bytes() / 2**20, 1) if strat.enabled else 0.0})
        enabled = strat.enabled
    if enabled and dev.type == "cuda" and not ps_on_cpu:
        comm_cfg["backend"] = "tfk_comm RCCL (own binding, librccl %s)" % _rccl_version()
        comm_cfg["rccl_transport"] = comm.transport_summary()
        comm_cfg["rccl_config"] = rccl_cfg
    loss = runner.last_loss()
    if runner.fallback:
        guards["capture_fallback"] = runner.fallback
    if gpu and hasattr(model, "rng_state"):
        # out-of-range events the bucketed embedding backward skipped (0: every step's counts valid)
        from tensorflow_k8s_amd.ops._lib import lib
        guards["emb_guard"] = int(lib().emb_guard_count())
    if wd is not None:
        guards["watchdog_s"] = wd.timeout_s
    comm_cfg["guards"] = guards
    bad = _numerics_failure(loss, guards.get("emb_guard", 0))
    if bad:
        # a corrupt run has no throughput: no metric line, non-zero exit
        print(json.dumps({"error": bad, "rank": rank, "model": args.model, "ms_per_step": round(ms, 3)}),
              file=sys.stderr, flush=True)
        if wd is not None:
            wd.exit_code = 0
        tfk_comm.shutdown()
        if wd is not None:
            wd.stop()
        return 3
    par = f"ps{len(ps_ranks)}+worker{nworkers}" if use_ps else f"dp{world}"
    if rank == worker_ranks[0] and not is_cnn:
        seq = model.cfg.seq_len if args.model.startswith("bert") else model.cfg.tgt_len
        toks = gb * (seq if args.model.startswith("bert") else model.cfg.src_len + model.cfg.tgt_len)
        print(json.dumps({
            "metric": f"{args.model} training throughput (whole node)", "value": round(toks / (ms / 1000.0), 1),
            "unit": "tokens/sec", "sequences_per_sec": round(value, 2), "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "step_ms": dist_ms, "per_rank_ms": per_rank,
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": _token_baseline(args.model, toks / (ms / 1000.0), nworkers),
            "dtype": "bf16+mxfp8" if args.fp8 else "bf16",
            "data": "synthetic token ids, random-init weights",
            "config": {"model": args.model, "global_batch": gb, "seq_len": seq, "per_gpu_batch": args.batch,
                       "parallelism": par, "strategy": strat_name,
                       "optimizer": opt_name, "hipgraph": runner.use_graph, "comm": comm_cfg},
            "loss": loss, **_update_report(model, master0)}), flush=True)
    elif rank == worker_ranks[0]:
        is_r50 = args.model == "resnet50"
        base = _baseline(nworkers) if is_r50 else None
        print(json.dumps({
            "metric": ("images/sec (whole node) ResNet-50 TFJob at 1/2/4/8 MI355X workers" if is_r50
                       else f"{args.model} images/sec (whole node)"),
            "value": round(value, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "step_ms": dist_ms, "per_rank_ms": per_rank,
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / base, 4) if base else None, "dtype": "bf16",
            "data": "synthetic (on-device ImageNet-shaped 224x224x3 bf16 batch, random-init weights)",
            "config": {"model": args.model, "global_batch": gb, "seq_len": None, "per_gpu_batch": args.batch,
                       "parallelism": par, "strategy": strat_name,
                       "optimizer": opt_name, "hipgraph": runner.use_graph, "comm": comm_cfg},
            "loss": loss, **_update_report(model, master0),
        }), flush=True)
    if wd is not None:
        wd.exit_code = 0  # the result is out: a hung teardown must not turn the run into a failure
    tfk_comm.shutdown()
    if wd is not None:
        wd.stop()


def _numerics_failure(loss, emb_guard: int) -> str | None:
    """Why the measured run is invalid (non-finite final loss, skipped embedding rows), else None."""
    import math
    if loss is not None and not math.isfinite(float(loss)):
        return f"non-finite loss {loss}"
    if emb_guard:
        return f"{emb_guard} out-of-range embedding events (emb_guard)"
    return None


def _update_report(model, master0) -> dict:
    if master0 is None:
        return {}
    d = (model.arena.master - master0).double()
    return {"update_norm": float(d.norm()), "update_sum": float(d.sum())}


def _rccl_version() -> str:
    from tensorflow_k8s_amd import _C
    v = _C.rccl_version()
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}"


def _gather_times(world_comm, cdev, world: int, mine_ms: float, worker_ranks=None):
    """MAX over ranks of the timed ms/step, and every worker's own value (all ranks must call)."""
    if world <= 1 or world_comm is None:
        return mine_ms, [round(mine_ms, 3)]
    t = torch.tensor([mine_ms], dtype=torch.float64, device=cdev)
    world_comm.all_reduce(t, op="max")
    g = torch.zeros(world, dtype=torch.float64, device=cdev)
    world_comm.all_gather(g, torch.tensor([mine_ms], dtype=torch.float64, device=cdev))
    vals = g.tolist()
    per = [round(vals[r], 3) for r in (worker_ranks if worker_ranks is not None else range(world))]
    return float(t.item()), per


def run_via_operator(args) -> int:
    """The headline metric measured the way BASELINE.json names it -- as a TFJob: start the native
    control plane (tfk-cluster: apiserver + operator + gang scheduler + kubelet), submit a TFJob of
    N one-GPU pods (Chief + N-1 Workers, amd.com/gpu: 1 each), and report the chief's JSON line.
    This process never initialises HIP; every GPU process is a kubelet-spawned pod."""
    import tempfile

    from tensorflow_k8s_amd.control.client import LocalCluster, tfjob_condition
    n = max(1, args.gpus)
    root = os.path.dirname(os.path.abspath(__file__))
    cmd = ["python3", os.path.join(root, "bench.py"), "--tfjob-worker", "--gpus", str(n), "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--model", args.model, "--bucket-mb", str(args.bucket_mb), "--comm-dtype", args.comm_dtype, "--graph",
           str(args.graph), "--fp8", str(args.fp8), "--strategy", args.strategy, "--ps-transport",
           args.ps_transport] + (["--batch", str(args.batch)] if args.batch else [])
    nps = args.ps if args.strategy == "ps" else 0
    if nps and n - nps < 1:
        raise SystemExit(f"--strategy ps needs --gpus > --ps ({n} <= {nps})")

    def rs(k, gpus=1):
        return {"replicas": k, "restartPolicy": "Never", "template": {"spec": {"containers": [{
            "name": "tensorflow", "image": "tfk/runtime", "command": cmd,
            "env": [{"name": "PYTHONPATH", "value": root}],
            "resources": {"limits": {"amd.com/gpu": gpus}}}]}}}
    # TF replica map: Chief + Workers compute; PS replicas (BASELINE config 3: PS=2/worker=6) own a
    # GPU on the rccl transport, none on the gloo (CPU parameter server) transport
    specs = {"Chief": rs(1)}
    if n - nps > 1:
        specs["Worker"] = rs(n - nps - 1)
    if nps:
        specs["PS"] = rs(nps, 0 if args.ps_transport == "gloo" else 1)
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
           "metadata": {"name": f"bench-{args.model}", "namespace": "default",
                        "annotations": {"scheduling.tfk.io/gang-visible-gpus": "true"}},
           "spec": {"tfReplicaSpecs": specs, "runPolicy": {"backoffLimit": 0, "cleanPodPolicy": "None"}}}
    with LocalCluster(gpus=n - (nps if args.ps_transport == "gloo" else 0),
                      root_dir=tempfile.mkdtemp(prefix="tfk-bench-")) as c:
        c.client.create(job)
        j = c.client.wait_tfjob(job["metadata"]["name"], timeout=1800)
        log = c.client.logs(f"bench-{args.model}-chief-0")
        if tfjob_condition(j) != "Succeeded":
            sys.stderr.write(log[-4000:] + "\n")
            raise SystemExit(f"bench TFJob ended {tfjob_condition(j)}: {j.get('status')}")
    line = [l for l in log.splitlines() if l.startswith("{") and '"metric"' in l][-1]
    out = json.loads(line)
    out["config"]["launcher"] = "TFJob via tfk-cluster (operator + gang scheduler + kubelet), one pod per GPU"
    print(json.dumps(out), flush=True)
    return 0


def _token_baseline(model: str, value: float, world: int):
    """value / the stock PyTorch comparator (tools/stock_transformer.py, profiles/comparators.json)."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "comparators.json")) as f:
            v = json.load(f).get(f"{model.replace('-', '_')}_bf16_stock_pytorch_1gpu_tok_s")
        return round(value / (v * world), 4) if v else None
    except Exception:
        return None


def _baseline(world: int):
    """Stock PyTorch-ROCm comparator (eager, MIOpen/hipBLASLt, channels_last bf16 autocast) measured
    on MI355X by tools/stock_resnet.py and recorded in profiles/comparators.json;
    scaled by world for weak scaling. None until measured."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "comparators.json")) as f:
            v = json.load(f).get("resnet50_bf16_stock_pytorch_1gpu_img_s")
        return v * world if v else None
    except Exception:
        return None


if __name__ == "__main__":
    sys.exit(main() or 0)
