"""tfk comm layer: RCCL (torch.distributed "nccl" on ROCm) collectives as the runtime uses them,
plus the two tools a multi-GPU MI355X job needs to trust its interconnect:

* a bus-bandwidth microbenchmark (all_reduce / all_gather / reduce_scatter / all_to_all /
  broadcast, nccl-tests conventions: algbw = bytes / time, busbw = algbw x the op's ring factor)
  -- ``python -m torch.distributed.run --nproc-per-node N -m tensorflow_k8s_amd.parallel.comm``;
* a transport report: RCCL is asked to log its channel setup (NCCL_DEBUG=INFO, subsystems INIT
  and P2P, to a per-process file) and the "via P2P/IPC | SHM | NET" lines are counted, so a run
  can show that its rings really ride xGMI peer-to-peer -- e.g. that per-pod HIP_VISIBLE_DEVICES
  isolation (one GPU visible per TFJob pod) did not push RCCL onto host shared memory.

xGMI on an 8x MI355X node is point-to-point (7 links x ~153 GB/s per GPU): a ring all-reduce is
bound by one link per hop, so the busbw reported here is what bucket sizing (parallel/mwms.py)
and the PS shard plan (parallel/ps.py) are tuned against.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import time

import torch
import torch.distributed as dist

# nccl-tests bus-bandwidth factors (per-rank bytes moved over the slowest link, relative to size)
def bus_factor(op: str, world: int) -> float:
    if world <= 1:
        return 1.0
    if op == "all_reduce":
        return 2.0 * (world - 1) / world
    if op in ("all_gather", "reduce_scatter", "all_to_all"):
        return (world - 1) / world
    return 1.0  # broadcast / reduce


_LOG_ENV = "TFK_RCCL_TRANSPORT_LOG"

RCCL_ALGOS = ("Ring", "Tree", "CollNet", "NVLS")
RCCL_PROTOS = ("Simple", "LL", "LL128")


def configure_rccl(algo: str | None = None, proto: str | None = None, min_channels: int = 0,
                   max_channels: int = 0) -> dict:
    """RCCL algorithm / protocol / channel control (NCCL_ALGO, NCCL_PROTO, NCCL_MIN/MAX_NCHANNELS),
    applied before the first communicator exists. On the fully connected 8x MI355X xGMI mesh one
    ring uses one outbound link per GPU: more channels (concurrent rings over different links) raise
    large-message bus bandwidth, LL/LL128 cut small-message latency. Returns the settings in force
    (for the bench record). Values already present in the environment are left alone."""
    want = {}
    if algo:
        if algo not in RCCL_ALGOS:
            raise ValueError(f"RCCL algorithm must be one of {RCCL_ALGOS}, got {algo}")
        want["NCCL_ALGO"] = algo
    if proto:
        if proto not in RCCL_PROTOS:
            raise ValueError(f"RCCL protocol must be one of {RCCL_PROTOS}, got {proto}")
        want["NCCL_PROTO"] = proto
    if min_channels:
        want["NCCL_MIN_NCHANNELS"] = str(int(min_channels))
    if max_channels:
        want["NCCL_MAX_NCHANNELS"] = str(int(max_channels))
    for k, v in want.items():
        os.environ.setdefault(k, v)
    return {k: os.environ[k] for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS")
            if k in os.environ}


def enable_transport_log(directory: str | None = None) -> str | None:
    """Ask RCCL to log channel/transport setup to <dir>/rccl.<host>.<pid>.log. Must run before the
    first communicator is created (RCCL reads its environment at comm init). A no-op when the user
    already configured NCCL_DEBUG. Returns the log directory."""
    if "NCCL_DEBUG" in os.environ:
        return None
    d = directory or os.environ.get("TMPDIR", "/tmp")
    os.makedirs(d, exist_ok=True)
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,P2P"
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "rccl.%h.%p.log")
    os.environ[_LOG_ENV] = d
    return d


_VIA = re.compile(r"via (P2P/IPC(?:/read)?|P2P/direct pointer|P2P/CUMEM|P2P|SHM(?:/direct)?|NET/\S+|COLLNET)")


def transport_summary(pid: int | None = None) -> dict:
    """Counts of RCCL channel connections by transport from this process's transport log."""
    d = os.environ.get(_LOG_ENV)
    if not d:
        return {}
    pid = os.getpid() if pid is None else pid
    out: dict[str, int] = {}
    for path in glob.glob(os.path.join(d, f"rccl.*.{pid}.log")):
        with open(path, errors="replace") as f:
            for line in f:
                m = _VIA.search(line)
                if m:
                    k = m.group(1)
                    out[k] = out.get(k, 0) + 1
    return out


def _make(op: str, nbytes: int, world: int, dtype: torch.dtype, dev):
    esz = torch.empty((), dtype=dtype).element_size()
    n = max(world, nbytes // esz // world * world)
    x = torch.ones(n, dtype=dtype, device=dev)
    if op == "all_reduce" or op == "broadcast":
        return (x,), n * esz
    if op == "all_gather":
        out = torch.empty(n, dtype=dtype, device=dev)
        return (out, x[: n // world]), n * esz
    if op == "reduce_scatter":
        out = torch.empty(n // world, dtype=dtype, device=dev)
        return (out, x), n * esz
    if op == "all_to_all":
        return (torch.empty_like(x), x), n * esz
    raise ValueError(f"unknown collective {op}")


def _call(op: str, args, group=None):
    if op == "all_reduce":
        return dist.all_reduce(args[0], group=group)
    if op == "broadcast":
        return dist.broadcast(args[0], 0, group=group)
    if op == "all_gather":
        return dist.all_gather_into_tensor(args[0], args[1], group=group)
    if op == "reduce_scatter":
        return dist.reduce_scatter_tensor(args[0], args[1], group=group)
    if op == "all_to_all":
        return dist.all_to_all_single(args[0], args[1], group=group)
    raise ValueError(op)


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def bench_collective(op: str, nbytes: int, iters: int = 20, warmup: int = 5, dtype=torch.bfloat16,
                     group=None) -> dict:
    """Time one collective at one size; the slowest rank's mean defines the result."""
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    args, size = _make(op, nbytes, world, dtype, dev)
    for _ in range(warmup):
        _call(op, args, group)
    _sync(dev)
    dist.barrier(group=group)
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        _call(op, args, group)
    _sync(dev)
    dt = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
    t = float(dt.item())
    algbw = size / t / 1e9
    return {"op": op, "bytes": size, "dtype": str(dtype).replace("torch.", ""), "world": world,
            "time_us": round(t * 1e6, 2), "algbw_GBps": round(algbw, 3),
            "busbw_GBps": round(algbw * bus_factor(op, world), 3)}


def _size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * mult[s[-1]]) if s[-1] in mult else int(s)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="RCCL bus-bandwidth microbenchmark (nccl-tests conventions)")
    ap.add_argument("--ops", default="all_reduce,all_gather,reduce_scatter,all_to_all,broadcast")
    ap.add_argument("--min-bytes", default="1M")
    ap.add_argument("--max-bytes", default="256M")
    ap.add_argument("--factor", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"])
    ap.add_argument("--transport-log", default="", help="directory for RCCL's transport log (default $TMPDIR)")
    ap.add_argument("--rccl-algo", default="", help="|".join(RCCL_ALGOS))
    ap.add_argument("--rccl-proto", default="", help="|".join(RCCL_PROTOS))
    ap.add_argument("--rccl-channels", type=int, default=0, help="NCCL_MIN_NCHANNELS")
    args = ap.parse_args(argv)
    rccl_cfg = configure_rccl(args.rccl_algo or None, args.rccl_proto or None, args.rccl_channels)
    backend = args.backend
    if backend == "auto":
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        enable_transport_log(args.transport_log or None)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    kw = {}
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    sizes, s = [], _size(args.min_bytes)
    while s <= _size(args.max_bytes):
        sizes.append(s)
        s *= max(2, args.factor)
    for op in args.ops.split(","):
        for nb in sizes:
            r = bench_collective(op, nb, args.iters, args.warmup, dtype)
            if rank == 0:
                print(json.dumps(r), flush=True)
    if rank == 0 and backend == "nccl":
        print(json.dumps({"rccl_transport": transport_summary(), "rccl_config": rccl_cfg}), flush=True)
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
