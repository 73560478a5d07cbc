"""Comm layer on CPU (gloo): MWMS bf16 wire buckets vs f32, in-order bucket launch, coalesced state
broadcast, and the bus-bandwidth microbenchmark (parallel/comm.py) at world size 2.
Reference behaviour: SURVEY §2 D3/D4 (MultiWorkerMirroredStrategy all-reduce), §5.8 (comm backend)."""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from conftest import ROOT, free_port
from test_runtime_cpu import BASE, _launch

PY = sys.executable


def test_mwms_bf16_wire_matches_f32(tmp_path, native_ext):
    """2-worker LeNet MWMS: the worker-mean loss trajectory with bf16 gradient buckets on the wire
    tracks the f32-wire trajectory (measured: <= 0.3 % over the first 6 steps, ~2 % after 12 SGD
    steps at lr 0.05) and is not bit-identical, so the bf16 path really ran."""
    traj = {}
    for dt in ("f32", "bf16"):
        p = free_port()
        r = _launch([("chief", 0), ("worker", 0)], {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"]},
                    BASE[:-1] + ["2", "--comm-dtype", dt], str(tmp_path))
        assert all(v[0] == 0 for v in r.values()), {k: v[2][-1500:] for k, v in r.items()}
        traj[dt] = [e["loss"] for e in r[("chief", 0)][1] if e.get("event") == "train"]
    a, b = traj["f32"], traj["bf16"]
    assert len(a) == len(b) == 6
    rel = [abs(x - y) / abs(x) for x, y in zip(a, b)]
    assert max(rel[:3]) <= 5e-3 and max(rel) <= 4e-2, traj
    assert a != b, traj


@pytest.fixture
def world1_gloo(tmp_path):
    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/store", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def _arena(n_params=6, numel=1000):
    from tensorflow_k8s_amd.runtime.arena import ParamArena, ParamSpec
    a = ParamArena()
    for i in range(n_params):
        a.add(ParamSpec(f"p{i}", (numel,), init="normal", decay=i % 2 == 0))
    a.add_buffer("moving_mean", torch.arange(5, dtype=torch.float32))
    a.add_buffer("moving_var", torch.ones(3, dtype=torch.float32))
    a.add_buffer("global_step", torch.zeros(1, dtype=torch.int64))
    return a.finalize("cpu")


def test_bucket_launch_order_is_rank_independent(world1_gloo):
    """Buckets launch strictly in bucket order whatever order gradients become ready, so every rank
    issues the same collective sequence; bf16 wire round-trips the grads into the f32 arena."""
    from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
    a = _arena()
    s = MultiWorkerMirroredStrategy(a, bucket_mb=1000 * 4 / 2**20, comm_dtype="bf16", force=True)
    assert s.enabled and len(s.buckets) >= 4
    launched = []
    orig = s._launch
    s._launch = lambda b: (launched.append(s.buckets.index(b)), orig(b))
    a.grad.copy_(torch.linspace(-3, 3, a.numel))
    want = a.grad.to(torch.bfloat16).float()
    s.begin_step()
    ps = sorted(a.params, key=lambda p: -p.offset)  # readiness in reverse bucket order
    a.grad_ready(*ps[:-1])
    assert launched == []  # bucket 0 not complete -> nothing may launch yet
    a.grad_ready(ps[-1])
    s.finish_step()
    assert launched == sorted(launched) and len(launched) == len(s.buckets)
    torch.testing.assert_close(a.grad, want, rtol=0, atol=0)
    assert s.wire_bytes() == sum(b.end - b.start for b in s.buckets) * 2


def test_broadcast_parameters_coalesces_buffers(world1_gloo):
    from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
    a = _arena()
    before = [b.tensor.clone() for b in a.buffers]
    s = MultiWorkerMirroredStrategy(a, force=True)
    calls = []
    real = dist.broadcast
    try:
        dist.broadcast = lambda t, *args, **kw: (calls.append(t.dtype), real(t, *args, **kw))[1]
        s.broadcast_parameters()
    finally:
        dist.broadcast = real
    assert calls.count(torch.float32) == 2 and calls.count(torch.int64) == 1  # arena + f32 buffers + i64
    for b, v in zip(a.buffers, before):
        assert torch.equal(b.tensor, v)
    assert torch.equal(a.compute, a.master.to(torch.bfloat16))


def test_comm_dtype_validation():
    from tensorflow_k8s_amd.parallel.mwms import comm_dtype_of
    assert comm_dtype_of("bf16") is torch.bfloat16 and comm_dtype_of(torch.float32) is torch.float32
    with pytest.raises(ValueError):
        comm_dtype_of("fp8")
    with pytest.raises(ValueError):
        comm_dtype_of(torch.float16)


def test_bus_factors():
    from tensorflow_k8s_amd.parallel.comm import bus_factor
    assert bus_factor("all_reduce", 8) == pytest.approx(1.75)
    assert bus_factor("all_gather", 8) == pytest.approx(0.875)
    assert bus_factor("broadcast", 8) == 1.0 and bus_factor("all_reduce", 1) == 1.0


def test_comm_bench_world2_gloo(tmp_path):
    """The busbw microbenchmark runs every collective at world size 2 (gloo) and reports rows with
    nccl-tests fields."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(free_port()), "-m", "tensorflow_k8s_amd.parallel.comm",
                        "--backend", "gloo", "--min-bytes", "64K", "--max-bytes", "1M", "--iters", "3", "--warmup", "1",
                        "--dtype", "f32"], env=env, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    ops = {x["op"] for x in rows}
    assert ops == {"all_reduce", "all_gather", "reduce_scatter", "all_to_all", "broadcast"}, ops
    for x in rows:
        assert x["world"] == 2 and x["time_us"] > 0 and x["busbw_GBps"] > 0
    ar = [x for x in rows if x["op"] == "all_reduce"][0]
    assert ar["busbw_GBps"] == pytest.approx(ar["algbw_GBps"], rel=1e-2)  # 2(n-1)/n = 1 at n=2


def test_transport_summary_parses_rccl_lines(tmp_path, monkeypatch):
    from tensorflow_k8s_amd.parallel import comm
    monkeypatch.setenv("TFK_RCCL_TRANSPORT_LOG", str(tmp_path))
    (tmp_path / f"rccl.host.{os.getpid()}.log").write_text(
        "host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n"
        "host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC\n"
        "host:1:1 [0] NCCL INFO Channel 02/0 : 0[0] -> 1[1] via SHM/direct/direct\n"
        "host:1:1 [0] NCCL INFO Connected all rings\n")
    assert comm.transport_summary() == {"P2P/IPC": 2, "SHM/direct": 1}


def test_collective_ps_plan_buckets(world1_gloo):
    """CollectivePlan buckets cover every parameter, never cross a shard or the decay/no-decay boundary,
    start and end on parameter boundaries, and respect the size cap."""
    from tensorflow_k8s_amd.parallel.ps import CollectivePlan, _param_spans, shard_bounds
    a = _arena(n_params=9, numel=3000)
    shards = shard_bounds(a.numel, 2, _param_spans(a))
    plan = CollectivePlan(a, shards, [0, 0], [0], bucket_mb=6000 * 4 / 2**20)
    bs = plan.buckets
    assert bs[0][0] == 0 and bs[-1][1] == a.numel
    for x, y in zip(bs, bs[1:]):  # contiguous, except over arena padding that holds no parameter
        assert x[1] == y[0] or not any(x[1] <= p.offset < y[0] for p in a.params), (x, y)
    starts = {p.offset for p in a.params} | {a.numel}
    nd = a.nodecay_region()[0]
    for lo, hi, s in bs:
        assert lo in starts or lo == nd
        slo, shi = shards[s]
        assert slo <= lo < hi <= shi
        assert not (lo < nd < hi)
        assert hi - lo <= 6000 + 3072  # cap + at most one more (aligned) parameter
    assert sum(plan._nparams) == len(a.params)
    assert set(plan.buckets_of(0)) | set(plan.buckets_of(1)) == set(range(len(bs)))


def test_configure_rccl_env(monkeypatch):
    from tensorflow_k8s_amd.parallel import comm
    for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS"):
        monkeypatch.delenv(k, raising=False)
    cfg = comm.configure_rccl("Ring", "LL128", min_channels=16)
    assert cfg == {"NCCL_ALGO": "Ring", "NCCL_PROTO": "LL128", "NCCL_MIN_NCHANNELS": "16"}
    monkeypatch.setenv("NCCL_ALGO", "Tree")  # user settings win
    assert comm.configure_rccl("Ring")["NCCL_ALGO"] == "Tree"
    with pytest.raises(ValueError):
        comm.configure_rccl("Butterfly")


TORCHRUN_SCRIPT = r"""
import hashlib, json, os, sys, torch
from tensorflow_k8s_amd.parallel import tfk_comm
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
store = tfk_comm.env_store(rank, world, timeout_s=60)
uid = tfk_comm.exchange_unique_id(store, rank, "world", lambda: os.urandom(128), 60)
c = tfk_comm.init(store, rank, world, torch.device("cpu"), 60)
x = torch.full((8,), float(rank + 1)); c.all_reduce(x)
mx = torch.tensor([float(rank)]); c.all_reduce(mx, op="max")
g = torch.zeros(world); c.all_gather(g, torch.tensor([float(rank * 10)]))
sub = c.split([0, 1], "pair"); y = torch.ones(3)
assert (sub is None) == (rank == 2)  # non-members get no sub-communicator
if sub is not None:
    sub.all_reduce(y)
c.barrier()
# one file per rank (3 ranks printing to one pipe can interleave inside a line)
with open(f"rank{rank}.json", "w") as f:
    f.write(json.dumps({"rank": rank, "uid": hashlib.sha1(uid).hexdigest(), "sum": x[0].item(), "max": mx.item(),
                        "gather": g.tolist(), "sub": y[0].item(), "backend": c.backend}))
tfk_comm.shutdown()
"""


def test_tfk_comm_bootstrap_under_torchrun(tmp_path):
    """bench.py's N-GPU bootstrap path on the CPU tier: under torchrun (the driver's launcher, whose
    agent hosts the store) every rank reaches the launcher's TCP store through env://, rank 0's
    unique id reaches all ranks unchanged, and the world communicator's collectives and a split
    sub-communicator work at world size 3."""
    script = tmp_path / "boot.py"
    script.write_text(TORCHRUN_SCRIPT)
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run([PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
                        "127.0.0.1", "--master-port", str(free_port()), str(script)], env=env, capture_output=True,
                       text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = sorted((json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(3)), key=lambda d: d["rank"])
    assert len(rows) == 3 and len({d["uid"] for d in rows}) == 1
    for d in rows:
        assert d["sum"] == 6.0 and d["max"] == 2.0 and d["gather"] == [0.0, 10.0, 20.0] and d["backend"] == "gloo"
    assert [d["sub"] for d in rows] == [2.0, 2.0, 1.0]


@pytest.mark.parametrize("extra,par", [([], "dp2"), (["--strategy", "ps", "--ps", "1", "--ps-transport", "rccl"], "ps1+worker1"),
                                       (["--strategy", "ps", "--ps", "1", "--ps-transport", "gloo"], "ps1+worker1")])
def test_bench_multi_rank_path_cpu_rehearsal(tmp_path, native_ext, extra, par):
    """bench.py's N-rank code path (torchrun bootstrap, world communicator, MWMS / both PS
    transports, barriers, MAX-over-ranks timing, per-rank gather, the one JSON line) rehearsed on
    the CPU tier with gloo and the fp32 executor -- the path the driver's multi-GPU run takes,
    minus the GPU. Not a measurement."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--cpu-rehearsal", "--model", "resnet50", "--batch", "2", "--steps", "1", "--warmup", "1"] + extra,
                       env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(lines) == 1, r.stdout[-2000:]  # exactly one rank prints
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == par and d["value"] > 0
    assert d["config"]["global_batch"] == (4 if par == "dp2" else 2)
    assert len(d["per_rank_ms"]) == (2 if par == "dp2" else 1)
