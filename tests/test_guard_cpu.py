"""CPU tests of the first-multi-GPU-run guards (runtime/guard.py, runtime/watchdog.py): unanimous
graph-or-eager agreement through the job store, the communicator self-test, the watchdog's RCCL
async-error polling, and a survivor whose peer stalls before the first collective."""
import json
import os
import subprocess
import sys

import pytest
import torch.distributed as dist

from conftest import ROOT, free_port
from tensorflow_k8s_amd.runtime.guard import Agreement, InjectedCaptureFault, capture_fault
from tensorflow_k8s_amd.runtime.watchdog import EXIT_RETRY

PY = sys.executable


def _torchrun(tmp_path, script: str, n: int, extra_env=None, timeout=240):
    p = tmp_path / "script.py"
    p.write_text(script)
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", **(extra_env or {}))
    return subprocess.run([PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(p)],
                          env=env, capture_output=True, text=True, timeout=timeout, cwd=str(tmp_path))


def test_agreement_single_process_and_hashstore():
    a = Agreement(None, 0, [0])
    assert a.decide("x", True) == (True, {})
    assert a.decide("x", False, "boom") == (False, {0: "boom"})
    # a store with every vote already present: the decision reads all of them
    st = dist.HashStore()
    b = Agreement(st, 0, [0, 1], timeout_s=5, prefix="t")
    st.set("t/cap/0/1", "err:rank one failed")
    ok, bad = b.decide("cap", True)
    assert not ok and bad == {1: "rank one failed"}
    assert b.log[-1] == {"decision": "cap", "ok": False, "failed_ranks": [1]}
    st.set("t/cap/1/1", "ok")  # the next decision of the same name uses a fresh key
    assert b.decide("cap", True) == (True, {})


def test_capture_fault_selector(monkeypatch):
    monkeypatch.setenv("TFK_FAULT_CAPTURE", "1")
    with pytest.raises(InjectedCaptureFault):
        capture_fault("probe", 3)
    capture_fault("step", 3)  # "1" means the probe only
    monkeypatch.setenv("TFK_FAULT_CAPTURE", "step")
    monkeypatch.setenv("TFK_FAULT_CAPTURE_RANK", "2")
    capture_fault("step", 1)
    with pytest.raises(InjectedCaptureFault):
        capture_fault("step", 2)


PROBE_SCRIPT = r"""
import json, os, torch
from tensorflow_k8s_amd.parallel import tfk_comm
from tensorflow_k8s_amd.runtime.guard import Agreement, capture_probe, comm_self_test
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
store = tfk_comm.env_store(rank, world, timeout_s=60)
c = tfk_comm.init(store, rank, world, torch.device("cpu"), 60)
st = comm_self_test(c)
agree = Agreement(c.store, rank, list(range(world)), timeout_s=60)
ok, why = capture_probe(c, agree, rank)
# a later, independent decision in which everyone succeeds
ok2, _ = agree.decide("step_capture", True)
with open(f"rank{rank}.json", "w") as f:
    f.write(json.dumps({"rank": rank, "self_test": st["ok"], "graph": ok, "why": why, "ok2": ok2, "log": agree.log}))
tfk_comm.shutdown()
"""


def test_one_rank_probe_failure_makes_all_three_ranks_eager(tmp_path):
    """3 ranks under torchrun (gloo): rank 1's injected capture-probe failure is published through
    the job store and every rank -- including the two whose probe succeeded -- chooses eager, with
    rank 1's reason; the communicator self-test passed first on all ranks."""
    r = _torchrun(tmp_path, PROBE_SCRIPT, 3, {"TFK_FAULT_CAPTURE": "probe", "TFK_FAULT_CAPTURE_RANK": "1"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(3)]
    for d in rows:
        assert d["self_test"] is True
        assert d["graph"] is False and "rank 1" in d["why"] and "injected probe capture failure" in d["why"]
        assert d["ok2"] is True
        assert d["log"][0] == {"decision": "probe_capture", "ok": False, "failed_ranks": [1]}


def test_probe_agreement_all_ok(tmp_path):
    r = _torchrun(tmp_path, PROBE_SCRIPT, 2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(2)]
    assert all(d["graph"] is True and d["why"] == "ok" for d in rows)
    assert [e["decision"] for e in rows[0]["log"]] == ["probe_capture", "probe_replay", "step_capture"]


def test_watchdog_fires_on_comm_async_error(tmp_path):
    """A communicator reporting an asynchronous error (ncclCommGetAsyncError) fires the watchdog
    on its next tick -- long before the heartbeat timeout -- aborts every live communicator and
    exits 143 with a comm_error event."""
    mark = tmp_path / "aborted"
    code = f"""
import time
from tensorflow_k8s_amd.parallel import tfk_comm
from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog
class Stub:
    tag = "world"
    def __init__(self): self.err = ""
    def async_error(self): return self.err
    def abort(self):
        open({str(mark)!r}, "a").write("aborted\\n"); return True
c = Stub(); tfk_comm._LIVE.add(c)
w = StepWatchdog(600, poll_s=0.05, comm_checks=True).start()
for step in range(4):
    w.beat(step); time.sleep(0.1)
c.err = "remote process exited or there was a network error"
time.sleep(30)
"""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([PY, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == EXIT_RETRY, r.stdout + r.stderr
    assert mark.read_text().split() == ["aborted"]
    evs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert evs[0]["kind"] == "comm_error" and "remote process exited" in evs[0]["message"]
    assert evs[0]["idle_s"] < 5


STALL_SCRIPT = r"""
import os, time, torch
from tensorflow_k8s_amd.parallel import tfk_comm
from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
store = tfk_comm.env_store(rank, world, timeout_s=60)
c = tfk_comm.init(store, rank, world, torch.device("cpu"), 120)
w = StepWatchdog(3.0, poll_s=0.1, name=f"rank{rank}", comm_checks=True).start()
w.beat(0, phase="first collective")
if rank == 1:
    for i in range(600):  # a stalled peer: alive (its own heartbeat keeps going), never joins
        w.beat(0); time.sleep(0.1)
x = torch.ones(4)
c.all_reduce(x)      # the survivor blocks here (gloo timeout 120 s) with the GIL released
print("unreachable", flush=True)
"""


def test_survivor_watchdog_fires_when_peer_stalls_before_first_collective(tmp_path):
    """a rank blocked in its first collective (peer alive but stalled) must not hold the
    GIL -- its watchdog thread fires after the heartbeat timeout and exits 143."""
    r = _torchrun(tmp_path, STALL_SCRIPT, 2, timeout=120)
    assert r.returncode != 0
    out = r.stdout + r.stderr
    assert "unreachable" not in out
    evs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"kind"' in l]
    assert evs and evs[0]["kind"] == "watchdog" and evs[0]["phase"] == "first collective", out[-3000:]
    assert "exitcode  : 143" in out or "exitcode: 143" in out or "143" in out


def test_bench_rehearsal_injected_probe_failure_runs_eager(tmp_path, native_ext):
    """bench.py at 2 ranks (CPU rehearsal): an injected capture-probe failure on rank 1 is reported
    in the JSON line (capture_probe names rank 1), the self-test result and the armed watchdog are
    recorded, and the run completes eagerly."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", TFK_FAULT_CAPTURE="1", TFK_FAULT_CAPTURE_RANK="1")
    r = subprocess.run([PY, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--cpu-rehearsal", "--model", "resnet50", "--batch", "2", "--steps", "1", "--warmup", "1"],
                       env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l][0]
    g = d["config"]["comm"]["guards"]
    assert g["comm_self_test"]["ok"] is True and g["watchdog_s"] == 300.0
    assert "rank 1" in g["capture_probe"] and "injected" in g["capture_probe"]
    assert d["config"]["hipgraph"] is False


def test_watchdog_follows_device_completion():
    """beat_device: while enqueued steps are pending, only their completion counts as progress --
    a device that stops completing fires the watchdog although the host keeps enqueuing (host
    beats no longer mask it); completed steps keep it quiet."""
    import time
    from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog

    class Ev:
        def __init__(self, done):
            self.done = done

        def query(self):
            return self.done
    fired = []
    w = StepWatchdog(0.5, on_timeout=lambda step, idle: fired.append((step, idle)), poll_s=0.05).start()
    try:
        for i in range(8):  # a healthy device: every enqueued step completes
            w.beat_device(i, Ev(True))
            time.sleep(0.1)
        assert not fired and w.device_step == 7
        stuck = Ev(False)
        w.beat_device(8, stuck)
        for i in range(9, 20):  # the host keeps enqueuing (and beating) behind a hung step
            w.beat_device(i, Ev(True))
            w.beat(i)
            time.sleep(0.1)
            if fired:
                break
        assert fired and fired[0][0] == 7, fired  # last COMPLETED step
    finally:
        w.stop()


def test_watchdog_poll_retires_by_identity_when_trimmed_concurrently():
    """A beat_device that trims the pending list while _poll_device queries its snapshot must not
    retire (or report as completed) a newer event that is still pending."""
    from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog
    w = StepWatchdog(60.0)
    w.MAX_PENDING = 3

    class Ev:
        def __init__(self, done, hook=None):
            self.done, self.hook = done, hook

        def query(self):
            if self.hook:
                self.hook()
            return self.done
    e2 = Ev(False)
    w.beat_device(0, Ev(True))
    w.beat_device(1, Ev(True, hook=lambda: w.beat_device(3, Ev(False))))  # trims entry 1 mid-poll
    w.beat_device(2, e2)
    w._poll_device()
    assert w.device_step == 0
    assert any(ev is e2 for _, ev in w._dev)
