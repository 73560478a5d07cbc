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
            "import time\nStepWatchdog(0.2, poll_s=0.02).start()\ntime.sleep(5)\n")
    env = dict(os.environ, TFK_TERMINATION_LOG=str(term), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == EXIT_RETRY, r.stderr
    assert "watchdog" in term.read_text()
    ev = json.loads(r.stdout.strip().splitlines()[-1])
    assert ev["kind"] == "watchdog"


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
