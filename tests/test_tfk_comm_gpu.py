"""tfk_comm -- the runtime's own RCCL binding (csrc/bindings/comm.cpp, parallel/tfk_comm.py) -- on one
MI355X: store bootstrap of the unique id, every collective against its closed form at world size 1,
ncclCommSplit sub-communicators, grouped send/recv, RCCL kernels captured inside a hipGraph and
replayed, and ncclCommAbort leaving a dead communicator that refuses further calls.
Multi-GPU rings are the driver's 8-GPU run; this pins the binding. Reference behaviour: SURVEY §2
D3 (comm backend), §5.3 (abort on failure), §5.8."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import json, os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["TFK_ROOT"])
from tensorflow_k8s_amd import _C
from tensorflow_k8s_amd.parallel import tfk_comm
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
out = {"version": _C.rccl_version()}
c = tfk_comm.init(dist.HashStore(), 0, 1, dev)
assert tfk_comm.world() is c and c.backend == "rccl" and (c.rank, c.world) == (0, 1)
x = torch.randn(1 << 20, device=dev)
y = x.clone(); c.all_reduce(y); out["all_reduce"] = bool(torch.equal(x, y))
yb = x.bfloat16(); c.all_reduce(yb, op="max"); out["all_reduce_bf16"] = bool(torch.equal(yb, x.bfloat16()))
o = torch.empty_like(x); c.all_reduce(x, out=o); out["out_of_place"] = bool(torch.equal(o, x))
b = x.clone(); c.broadcast(b, 0); out["broadcast"] = bool(torch.equal(b, x))
r = x.clone(); c.reduce(r, 0); out["reduce"] = bool(torch.equal(r, x))
g = torch.empty_like(x); c.all_gather(g, x); out["all_gather"] = bool(torch.equal(g, x))
rs = torch.empty_like(x); c.reduce_scatter(rs, x); out["reduce_scatter"] = bool(torch.equal(rs, x))
a2a = torch.empty_like(x); c.all_to_all(a2a, x); out["all_to_all"] = bool(torch.equal(a2a, x))
# grouped send/recv to self (one fused launch)
dst = torch.empty_like(x)
with c.group() as grp:
    grp.send(x, 0); grp.recv(dst, 0)
grp.handle.wait(); out["sendrecv"] = bool(torch.equal(dst, x))
# sub-communicator
sub = c.split([0], "sub"); s2 = x.clone(); sub.all_reduce(s2, op="sum")
out["split"] = bool(torch.equal(s2, x)) and sub.world == 1
# async handle: the current stream waits on the comm stream, no host block
h = c.all_reduce(y, async_op=True); h.wait(); torch.cuda.synchronize(); out["async"] = True
# capture: scale-then-all-reduce replayed 3x, the all-reduce node really re-runs each replay
buf = torch.ones(4096, device=dev); acc = torch.zeros(4096, device=dev)
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        t = buf * 2.0; c.all_reduce(t); acc.add_(t)
torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
acc.zero_()
gph = torch.cuda.CUDAGraph()
with torch.cuda.graph(gph):
    t = buf * 2.0
    hh = c.all_reduce(t, async_op=True)
    hh.wait()
    acc.add_(t)
for _ in range(3):
    gph.replay()
torch.cuda.synchronize()
out["graph"] = float(acc[0].item())
out["async_error"] = c.async_error()
# abort: the communicator is dead afterwards and says so
assert tfk_comm.abort_all() >= 1
out["aborted_valid"] = c._c.valid
try:
    c.all_reduce(y); out["after_abort"] = "no error"
except RuntimeError as e:
    out["after_abort"] = "aborted" in str(e)
print(json.dumps(out))
"""


def test_tfk_comm_world1_collectives_capture_abort():
    env = dict(os.environ, TFK_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["version"] >= 22600, out
    for k in ("all_reduce", "all_reduce_bf16", "out_of_place", "broadcast", "reduce", "all_gather", "reduce_scatter",
              "all_to_all", "sendrecv", "split", "async"):
        assert out[k] is True, (k, out)
    assert out["graph"] == 6.0, out  # 3 replays x (1 * 2.0) all-reduced over one rank
    assert out["async_error"] == "", out
    assert out["aborted_valid"] is False and out["after_abort"] is True, out
