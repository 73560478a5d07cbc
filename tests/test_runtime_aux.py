"""CPU tests of the runtime's auxiliary subsystems: step watchdog (failure detection) and the
Chrome-trace / roctx tracer."""
import json
import os
import subprocess
import sys
import threading
import time

from tensorflow_k8s_amd.runtime.watchdog import EXIT_RETRY, StepWatchdog
from tensorflow_k8s_amd.utils.tracing import Tracer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_watchdog_fires_without_heartbeat():
    hit = threading.Event()
    seen = {}

    def on_timeout(step, idle):
        seen.update(step=step, idle=idle)
        hit.set()

    wd = StepWatchdog(0.2, on_timeout=on_timeout, poll_s=0.02).start()
    wd.beat(7)
    assert hit.wait(2.0)
    assert wd.fired and seen["step"] == 7 and seen["idle"] > 0.2
    wd.stop()


def test_watchdog_quiet_while_beating():
    fired = threading.Event()
    with StepWatchdog(0.3, on_timeout=lambda s, i: fired.set(), poll_s=0.02) as wd:
        for i in range(15):
            wd.beat(i)
            time.sleep(0.05)
    assert not fired.is_set()


def test_watchdog_default_exits_retryable(tmp_path):
    """The default action exits the process with the operator-retryable code and writes the
    termination message."""
    term = tmp_path / "term"
    code = ("from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog\n"
            "import time\nStepWatchdog(0.2, poll_s=0.02).start()\ntime.sleep(60)\n")
    env = dict(os.environ, TFK_TERMINATION_LOG=str(term), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == EXIT_RETRY, r.stderr
    assert "watchdog" in term.read_text()
    evs = [json.loads(l) for l in r.stdout.strip().splitlines() if l.startswith("{")]
    assert evs[0]["kind"] == "watchdog"
    assert evs[-1] == {"event": "comm_aborted", "communicators": 0}


def test_watchdog_aborts_live_communicators_then_exits_143(tmp_path):
    """The watchdog path tears the rank's communicators down before exiting: every communicator
    registered with tfk_comm (RcclComm registers itself at construction) gets abort() -- the
    ncclCommAbort of the native binding -- and the process exits with the retryable 143. Here the
    registered communicators are stand-ins that record the call (no GPU in the CPU tier); the
    native abort itself is exercised on the MI355X by tests/test_tfk_comm_gpu.py."""
    mark = tmp_path / "aborted"
    code = f"""
import time
from tensorflow_k8s_amd.parallel import tfk_comm
from tensorflow_k8s_amd.runtime.watchdog import StepWatchdog
class Stub:
    def __init__(self, name): self.name = name
    def abort(self):
        with open({str(mark)!r}, "a") as f: f.write(self.name + "\\n")
        return True
keep = [Stub("world"), Stub("ps0/reduce")]
for c in keep: tfk_comm._LIVE.add(c)
w = StepWatchdog(0.3, poll_s=0.02).start()
for step in range(3):      # progress, then a 'hung collective'
    w.beat(step); time.sleep(0.05)
time.sleep(10)
"""
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == EXIT_RETRY, r.stderr
    assert sorted(mark.read_text().split()) == ["ps0/reduce", "world"]
    evs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert evs[0]["kind"] == "watchdog" and evs[0]["step"] == 2
    assert evs[-1] == {"event": "comm_aborted", "communicators": 2}


def test_tracer_chrome_trace(tmp_path):
    tr = Tracer(rank=3)
    with tr.span("step", step=1):
        with tr.span("forward"):
            time.sleep(0.01)
    tr.instant("checkpoint", step=1)
    path = tr.dump(str(tmp_path / "t.json"))
    d = json.load(open(path))
    names = [e["name"] for e in d["traceEvents"]]
    assert "step" in names and "forward" in names and "checkpoint" in names
    fwd = next(e for e in d["traceEvents"] if e["name"] == "forward")
    step = next(e for e in d["traceEvents"] if e["name"] == "step")
    assert fwd["pid"] == 3 and fwd["dur"] >= 9000 and step["dur"] >= fwd["dur"]
    assert step["ts"] <= fwd["ts"]


def test_tracer_disabled_is_noop(tmp_path):
    tr = Tracer(enabled=False)
    with tr.span("x"):
        pass
    assert tr.events == []


def test_dropout_rate_quantization_is_validated():
    """the kernels' 8-bit mask threshold applies round(256 p) / 256; unrepresentable
    rates are rejected instead of silently changing meaning."""
    import pytest
    from tensorflow_k8s_amd.models.bert import BertConfig
    from tensorflow_k8s_amd.models.transformer import TransformerConfig
    from tensorflow_k8s_amd.ops.elementwise import check_rate, effective_rate
    assert abs(effective_rate(0.1) - 26 / 256) < 1e-12 and check_rate(0.1) == 0.1
    assert effective_rate(0.0) == 0.0 and check_rate(0.0) == 0.0
    for bad in (1e-4, 0.999, 1.0, -0.1):
        with pytest.raises(ValueError):
            check_rate(bad)
    with pytest.raises(ValueError):
        TransformerConfig(dropout=0.9995)
    with pytest.raises(ValueError):
        BertConfig(attn_dropout=1e-3)


def test_bench_refuses_corrupt_runs():
    """bench.py prints no metric line (exit 3) for a non-finite final loss or skipped embedding rows."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b._numerics_failure(2.5, 0) is None
    assert b._numerics_failure(None, 0) is None
    assert "non-finite" in b._numerics_failure(float("nan"), 0)
    assert "non-finite" in b._numerics_failure(float("inf"), 0)
    assert "emb_guard" in b._numerics_failure(2.5, 3)
