"""TF_CONFIG cluster resolver (TFConfigClusterResolver equivalent).

The operator injects TF_CONFIG = {"cluster": {"chief": [...], "worker": [...], "ps": [...]},
"task": {"type": ..., "index": ...}, "environment": "cloud"} (v1alpha1 uses "master" for the
chief). Rank layout of the training world (one process per GPU):
    rank 0            chief / master (or worker 0 when the job has no chief)
    ranks 1..         workers (in index order)
    then              parameter servers (ParameterServerStrategy)
    evaluator         NOT part of the world (rank -1), it only reads checkpoints.
The rendezvous address is the chief's "host:port" (port = tfPort, default 2222). Under the
single-node emulation (TFK_LOCAL_DNS=1) "<svc>.<ns>.svc[...]" hostnames resolve to 127.0.0.1.
Falls back to torchrun variables (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT) or a single process.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field


@dataclass
class ClusterInfo:
    task_type: str = "worker"
    task_index: int = 0
    rank: int = 0
    world_size: int = 1
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    cluster: dict = field(default_factory=dict)
    worker_ranks: list = field(default_factory=list)  # ranks that compute (chief + workers)
    ps_ranks: list = field(default_factory=list)
    source: str = "local"

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @property
    def is_evaluator(self) -> bool:
        return self.task_type == "evaluator"

    @property
    def is_ps(self) -> bool:
        return self.task_type == "ps"

    @property
    def num_workers(self) -> int:
        return len(self.worker_ranks)


def _host_port(addr: str, local_dns: bool):
    host, _, port = addr.rpartition(":")
    if not host:
        host, port = addr, "2222"
    if local_dns and (".svc" in host or host.endswith(".local") or "." not in host):
        host = "127.0.0.1"
    return host, int(port)


def resolve(env: dict | None = None) -> ClusterInfo:
    env = dict(os.environ if env is None else env)
    local_dns = env.get("TFK_LOCAL_DNS", "0") == "1"
    if env.get("TF_CONFIG"):
        cfg = json.loads(env["TF_CONFIG"])
        cluster = {k.lower(): list(v) for k, v in cfg.get("cluster", {}).items()}
        task = cfg.get("task", {})
        ttype, tidx = task.get("type", "worker").lower(), int(task.get("index", 0))
        chief_key = "chief" if "chief" in cluster else ("master" if "master" in cluster else None)
        order = []
        if chief_key:
            order += [(chief_key, i) for i in range(len(cluster[chief_key]))]
        order += [("worker", i) for i in range(len(cluster.get("worker", [])))]
        order += [("ps", i) for i in range(len(cluster.get("ps", [])))]
        info = ClusterInfo(task_type=ttype, task_index=tidx, cluster=cluster, source="TF_CONFIG",
                           world_size=len(order))
        info.worker_ranks = [r for r, (t, _) in enumerate(order) if t != "ps"]
        info.ps_ranks = [r for r, (t, _) in enumerate(order) if t == "ps"]
        if ttype == "evaluator":
            info.rank = -1
        else:
            try:
                info.rank = order.index((ttype, tidx))
            except ValueError as e:
                raise ValueError(f"task {ttype}:{tidx} not in TF_CONFIG cluster {sorted(cluster)}") from e
        head = cluster[chief_key][0] if chief_key else (cluster.get("worker") or ["127.0.0.1:2222"])[0]
        info.master_addr, info.master_port = _host_port(head, local_dns)
        return info
    if "WORLD_SIZE" in env and "RANK" in env:
        w, r = int(env["WORLD_SIZE"]), int(env["RANK"])
        return ClusterInfo(task_type="chief" if r == 0 else "worker", task_index=r, rank=r, world_size=w,
                           master_addr=env.get("MASTER_ADDR", "127.0.0.1"), master_port=int(env.get("MASTER_PORT", 29500)),
                           worker_ranks=list(range(w)), source="torchrun")
    return ClusterInfo(worker_ranks=[0], source="local")


def make_store(info: ClusterInfo, timeout_s: float = 600.0, retries: int = 5):
    """The job's rendezvous store: torch's C++ TCPStore hosted by the chief on its tfPort. A
    port-in-use at the chief (k8s-operator.md:5 failure mode, typically the previous restart
    generation still shutting down) is retried, then reported as a retryable exit so the operator
    restarts the gang."""
    import datetime
    import time

    import torch.distributed as dist
    last = None
    for attempt in range(retries):
        try:
            return dist.TCPStore(info.master_addr, info.master_port, info.world_size, info.rank == 0,
                                 timeout=datetime.timedelta(seconds=timeout_s))
        except (RuntimeError, OSError) as e:
            last = e
            msg = str(e).lower()
            if "address already in use" in msg or "eaddrinuse" in msg:
                time.sleep(2.0 * (attempt + 1))
                continue
            raise
    raise RendezvousError(f"rendezvous at {info.master_addr}:{info.master_port} failed: port already in use ({last})")


def init_comm(info: ClusterInfo, device, backend: str = "auto", timeout_s: float = 600.0, retries: int = 5):
    """Rendezvous on the chief's store and create the world communicator (parallel/tfk_comm):
    ``rccl`` = the runtime's own RCCL communicator (GPU ranks), ``gloo`` = torch.distributed gloo
    (CPU ranks, CPU parameter servers). Returns None for a single process / the evaluator."""
    import torch

    from . import tfk_comm
    if info.world_size <= 1 or info.rank < 0:
        return None
    if backend == "auto":
        backend = "rccl" if torch.device(device).type == "cuda" else "gloo"
    store = make_store(info, timeout_s, retries)
    dev = torch.device(device) if backend == "rccl" else torch.device("cpu")
    return tfk_comm.init(store, info.rank, info.world_size, dev, timeout_s)


def init_process_group(info: ClusterInfo, backend: str, timeout_s: float = 600.0, retries: int = 5, device_id=None):
    """torch.distributed world on the chief's store (gloo tier and tools)."""
    import datetime

    import torch.distributed as dist
    if info.world_size <= 1 or info.rank < 0:
        return False
    store = make_store(info, timeout_s, retries)
    kw = {"device_id": device_id} if device_id is not None else {}
    dist.init_process_group(backend, store=store, rank=info.rank, world_size=info.world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return True


class RendezvousError(RuntimeError):
    exit_code = 143  # retryable by the operator's ExitCode policy
