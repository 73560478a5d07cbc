"""The collective parameter-server OWNER loop on one MI355X (parallel/ps.py ParameterServer.serve_steps /
_capture_owner): the path BASELINE config 3's two GPU parameter servers run. A world-1 tfk_comm RCCL
communicator with ps_ranks = worker_ranks = [0], several buckets per shard, AdamW and LAMB with
weight decay and a warmup + cosine schedule on the device (Optimizer.enable_device_schedule). The owner
runs OWNER_WARMUP eager steps, captures its step once and replays it; the result must equal an
owner that never captures (host schedule, eager every step): master weights, every slot and the
step counter after 8 steps, and the captured run must really have replayed a graph (owner_graph).

A fixed non-zero gradient is added to each bucket right before its reduce (inside the captured
step), so the update is not weight decay alone. Reference: SURVEY §2.2 D5, k8s-operator.md:6."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import json, os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["TFK_ROOT"])
from tensorflow_k8s_amd.parallel import tfk_comm, ps as PS
from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining
from tensorflow_k8s_amd.runtime.optimizer import AdamW, LAMB, LRSchedule
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
c = tfk_comm.init(dist.HashStore(), 0, 1, dev)
out = {}
for name, cls in (("adamw", AdamW), ("lamb", LAMB)):
    res = {}
    for capture in (False, True):
        PS.CAPTURE_OWNER = capture
        m = BertForPreTraining(BertConfig.tiny()).to(dev, seed=3)
        a = m.arena
        opt = cls(a, LRSchedule(1e-3, warmup=3, total=8, kind="cosine", end_lr=1e-4), weight_decay=0.01)
        srv = PS.ParameterServer(a, opt, 0, [0], [0])
        srv.setup_collective(bucket_mb=0.25, comm=c)
        g = torch.Generator(device=dev); g.manual_seed(7)
        G = torch.randn(a.numel, device=dev, generator=g) * 1e-2
        plan = srv._plan
        orig = plan.reduce
        def red(i, grad, deps=(), orig=orig, G=G, plan=plan):
            lo, hi, _ = plan.buckets[i]
            grad[lo:hi].add_(G[lo:hi])
            return orig(i, grad, deps)
        plan.reduce = red
        srv.serve_steps(0, 8)
        torch.cuda.synchronize()
        res[capture] = (a.master.clone(), {s: a.slot(s).clone() for s in opt.slot_names}, opt.sync_step(),
                        srv.owner_graph, srv.capture_fallback, len(plan.buckets_of(0)))
    e, g_ = res[False], res[True]
    diff = float((e[0] - g_[0]).abs().max())
    sdiff = max(float((e[1][s] - g_[1][s]).abs().max()) for s in e[1])
    out[name] = {"master_diff": diff, "slot_diff": sdiff, "steps": [e[2], g_[2]], "owner_graph": [e[3], g_[3]],
                 "fallback": g_[4], "buckets": g_[5], "slot_norm": float(sum(v.norm() for v in g_[1].values()))}
print("RESULT " + json.dumps(out))
"""


def test_captured_ps_owner_matches_eager_owner(tmp_path):
    env = dict(os.environ, TFK_ROOT=ROOT, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    for name, d in res.items():
        assert d["owner_graph"] == [False, True], (name, d)
        assert d["fallback"] == "", (name, d)
        assert d["buckets"] > 1, (name, d)  # several region updates per global step
        assert d["steps"] == [8, 8], (name, d)
        assert d["slot_norm"] > 0, (name, d)
        assert d["master_diff"] <= 1e-6 and d["slot_diff"] <= 1e-6, (name, d)
