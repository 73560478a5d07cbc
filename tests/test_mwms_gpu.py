"""MWMS over tfk_comm (the runtime's own RCCL communicator) on one MI355X: a world-size-1
communicator with forced collectives runs the real RCCL all-reduce path (bf16 wire buckets,
in-order launch on the comm stream, unpack) eagerly and captured in a hipGraph -- with the
weight-gradient side streams active in BOTH modes -- and both agree with the no-comm step (an
all-reduce over one rank is the identity up to the bf16 wire rounding). Multi-GPU rings are the
driver's 8-GPU run; this pins the code path the N-GPU bench replays.
Reference behaviour: SURVEY §2 D4 (MWMS), D6 (graph executor)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import os, sys, json, torch, torch.distributed as dist
os.environ["TFK_CONCURRENT_WGRAD"] = "1"   # side-stream weight gradients in eager steps too
sys.path.insert(0, os.environ["TFK_ROOT"])
from tensorflow_k8s_amd.models.resnet import ResNet, synthetic_imagenet
from tensorflow_k8s_amd.parallel import tfk_comm
from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
from tensorflow_k8s_amd.runtime import streams
from tensorflow_k8s_amd.runtime.optimizer import SGD
from tensorflow_k8s_amd.runtime.trainer import StepRunner
assert streams.MODE == "1"
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
comm = tfk_comm.init(dist.HashStore(), 0, 1, dev)
out = {}
for mode in ("nocomm", "eager", "graph"):
    m = ResNet(50, stages=[1, 1, 1, 1], num_classes=100).to(dev, seed=7)
    opt = SGD(m.arena, lr=0.05, momentum=0.9)
    s = MultiWorkerMirroredStrategy(m.arena, comm=comm if mode != "nocomm" else None, bucket_mb=2.0,
                                    comm_dtype="bf16", force=mode != "nocomm")
    s.configure_optimizer(opt)
    s.broadcast_parameters()
    x, y = synthetic_imagenet(16, dev, num_classes=100, seed=3)
    r = StepRunner(m, opt, s, (x, y), use_graph=mode == "graph")
    for _ in range(6):
        r.step()
    torch.cuda.synchronize()
    out[mode] = {"loss": r.last_loss(), "buckets": len(s.buckets), "enabled": s.enabled, "side": len(streams._side),
                 "w": m.arena.master.double().sum().item(), "wabs": m.arena.master.abs().double().sum().item()}
    torch.save(m.arena.master.cpu(), os.environ["TFK_OUT"] + "." + mode)
tfk_comm.shutdown()
print(json.dumps(out))
"""


def test_rccl_mwms_eager_and_graph_match_nocomm(tmp_path):
    env = dict(os.environ, TFK_ROOT=ROOT, TFK_OUT=str(tmp_path / "w"))
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json

    import torch
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["eager"]["enabled"] and out["graph"]["enabled"] and not out["nocomm"]["enabled"]
    assert out["eager"]["buckets"] > 3
    assert out["eager"]["side"] >= 1  # the eager run really forked weight gradients onto side streams
    ref = torch.load(str(tmp_path / "w.nocomm"), weights_only=True)
    for mode in ("eager", "graph"):
        w = torch.load(str(tmp_path / f"w.{mode}"), weights_only=True)
        cos = torch.nn.functional.cosine_similarity((w - ref).double().flatten(), ref.double().flatten(), dim=0)
        rel = (w - ref).norm() / ref.norm()
        # bf16 wire rounding of 6 steps of gradients: tiny drift, no structural difference
        assert rel < 2e-3, (mode, float(rel), float(cos))
        assert abs(out[mode]["loss"] - out["nocomm"]["loss"]) < 0.05 * abs(out["nocomm"]["loss"]), out
    wg, we = (torch.load(str(tmp_path / f"w.{m}"), weights_only=True) for m in ("graph", "eager"))
    assert (wg - we).norm() / we.norm() < 2e-3


PS_SCRIPT = r"""
import os, sys, json, torch, torch.distributed as dist
sys.path.insert(0, os.environ["TFK_ROOT"])
from tensorflow_k8s_amd.models.resnet import ResNet, synthetic_imagenet
from tensorflow_k8s_amd.parallel import tfk_comm
from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
from tensorflow_k8s_amd.parallel.ps import ParameterServerStrategy
from tensorflow_k8s_amd.runtime.optimizer import SGD
from tensorflow_k8s_amd.runtime.trainer import StepRunner
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
comm = tfk_comm.init(dist.HashStore(), 0, 1, dev)
out = {}
for mode in ("mwms", "ps_eager", "ps_graph"):
    m = ResNet(50, stages=[1, 1, 1, 1], num_classes=100).to(dev, seed=7)
    opt = SGD(m.arena, lr=0.05, momentum=0.9)
    if mode == "mwms":
        s = MultiWorkerMirroredStrategy(m.arena, comm=comm, bucket_mb=2.0, comm_dtype="bf16", force=True)
    else:
        s = ParameterServerStrategy(m.arena, [0], [0], "sync", transport="rccl", bucket_mb=2.0, comm=comm,
                                    wire_dtype=torch.bfloat16)
    s.configure_optimizer(opt)
    s.broadcast_parameters()
    x, y = synthetic_imagenet(16, dev, num_classes=100, seed=3)
    r = StepRunner(m, opt, s, (x, y), use_graph=mode != "ps_eager")
    for _ in range(6):
        r.step()
    torch.cuda.synchronize()
    out[mode] = {"loss": r.last_loss(), "graph": r.use_graph,
                 "buckets": len(s.plan.buckets) if mode != "mwms" else len(s.buckets)}
    torch.save(m.arena.master.cpu(), os.environ["TFK_OUT"] + "." + mode)
tfk_comm.shutdown()
print(json.dumps(out))
"""


def test_colocated_collective_ps_matches_forced_mwms(tmp_path):
    """the collective PS transport on GPU tensors -- bucketed bf16 reduce to the owner,
    unpack, per-bucket fused optimizer (step_region), broadcast of the bf16 compute copy -- with the
    owner colocated on worker 0 of a world-size-1 RCCL communicator, eager and hipGraph-captured,
    tracks forced-comm MWMS over 6 steps within bf16 wire tolerance."""
    env = dict(os.environ, TFK_ROOT=ROOT, TFK_OUT=str(tmp_path / "w"))
    r = subprocess.run([sys.executable, "-c", PS_SCRIPT], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json

    import torch
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["ps_graph"]["graph"] is True and out["ps_eager"]["graph"] is False and out["ps_eager"]["buckets"] > 3
    ref = torch.load(str(tmp_path / "w.mwms"), weights_only=True)
    for mode in ("ps_eager", "ps_graph"):
        w = torch.load(str(tmp_path / f"w.{mode}"), weights_only=True)
        rel = (w - ref).norm() / ref.norm()
        assert rel < 3e-3, (mode, float(rel))
        assert abs(out[mode]["loss"] - out["mwms"]["loss"]) < 0.05 * abs(out["mwms"]["loss"]), out
