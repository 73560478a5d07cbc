"""Step-progress watchdog: the runtime half of failure detection.

A collective whose peer died never returns: RCCL (and gloo) block inside the all-reduce until their
own timeout, which is minutes by default, and a wedged rank keeps its GPU busy. The watchdog is a
daemon thread that expects a heartbeat (``beat(step)``) at least every ``timeout_s`` seconds once
training has started. When the heartbeat stops it writes the termination message, logs one JSON
event, aborts every live tfk_comm RCCL communicator (``ncclCommAbort``: the rank's outstanding RCCL
kernels exit instead of spinning on a dead peer) and exits with 143, the retryable code of the operator's ExitCode restart policy: the
operator bumps the restart generation, every rank re-rendezvouses and training resumes from the
latest checkpoint (runtime/train.py, runtime/checkpoint.py).

Device-side progress: a replayed hipGraph returns to the host at once, so a host heartbeat after
``runner.step()`` only says the step was ENQUEUED. ``beat_device(step, event)`` (an event recorded
after the step) makes the watchdog follow completion instead: while enqueued steps are pending,
the clock runs from the last one the device finished, so a kernel or collective that hangs on the
device fires the watchdog after ``timeout_s`` even though the host keeps enqueuing (until HIP's
queue back-pressure blocks it) -- not only once the host itself stalls.

Besides the heartbeat, every tick polls the registered health checks -- by default
``tfk_comm.async_errors()`` (ncclCommGetAsyncError of every live communicator): a peer that RCCL has
already declared lost fires the watchdog at once instead of after the heartbeat timeout. The
multi-rank runtimes (bench.py, runtime/train.py) arm it by default at world size > 1.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

EXIT_RETRY = 143


class StepWatchdog:
    def __init__(self, timeout_s: float, on_timeout=None, poll_s: float | None = None, name: str = "train",
                 checks=None, comm_checks: bool = False):
        if timeout_s <= 0:
            raise ValueError("watchdog timeout must be > 0")
        self.timeout_s = float(timeout_s)
        self.poll_s = float(poll_s) if poll_s else min(1.0, self.timeout_s / 4)
        self.name = name
        self.on_timeout = on_timeout or self._default_timeout
        # health checks polled every tick: callables returning "" (healthy) or an error message
        self.checks = list(checks or [])
        if comm_checks:
            self.checks.append(comm_async_error)
        self.exit_code = EXIT_RETRY  # set to 0 once the job's result is out (a hung teardown is not a failure)
        self.phase = "train"
        self.error = ""
        self.last_step = -1
        self._last = time.monotonic()
        self._dev = []        # [(step, event)] enqueued steps whose completion is not yet seen
        self.device_step = -1
        self._stop = threading.Event()
        self._fired = threading.Event()
        self._lock = threading.Lock()
        self._thread = None

    # ------------------------------------------------------------------ control
    def start(self) -> "StepWatchdog":
        self._last = time.monotonic()
        self._thread = threading.Thread(target=self._run, name=f"tfk-watchdog-{self.name}", daemon=True)
        self._thread.start()
        return self

    def beat(self, step: int | None = None, phase: str | None = None) -> None:
        with self._lock:
            if not self._dev:  # while device steps are pending, only their completion is progress
                self._last = time.monotonic()
                if step is not None:
                    self.last_step = step
            if phase is not None:
                self.phase = phase

    MAX_PENDING = 256

    def beat_device(self, step: int, event, phase: str | None = None) -> None:
        """Step `step` was enqueued and `event` recorded after it (anything with .query())."""
        with self._lock:
            if not self._dev:
                self._last = time.monotonic()  # the device clock starts at the first pending step
            self._dev.append((step, event))
            if len(self._dev) > self.MAX_PENDING:
                del self._dev[1:len(self._dev) - self.MAX_PENDING + 1]  # keep the oldest
            if phase is not None:
                self.phase = phase

    def _poll_device(self) -> None:
        with self._lock:
            pend = list(self._dev)
        done = 0
        for st, ev in pend:
            try:
                ok = ev.query()
            except Exception:  # noqa: BLE001 -- a failed query is not progress
                ok = False
            if not ok:
                break
            done += 1
        if done:
            with self._lock:
                # retire by identity: beat_device may have trimmed the middle of the list since the
                # snapshot, so a positional prefix could name newer, still-pending events
                last = None
                for ent in pend[:done]:
                    if self._dev and self._dev[0] is ent:
                        last = self._dev.pop(0)
                if last is not None:
                    self.device_step = self.last_step = last[0]
                    self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5.0)

    @property
    def fired(self) -> bool:
        return self._fired.is_set()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    # ------------------------------------------------------------------ loop
    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            if self._dev:
                self._poll_device()
            with self._lock:
                idle = time.monotonic() - self._last
                step = self.last_step
            err = ""
            for chk in self.checks:
                try:
                    err = chk() or ""
                except Exception as e:  # a failing check is itself an error signal
                    err = f"{getattr(chk, '__name__', 'check')}: {e}"
                if err:
                    break
            if err or idle > self.timeout_s:
                self.error = err
                self._fired.set()
                self.on_timeout(step, idle)
                return

    def _default_timeout(self, step: int, idle: float) -> None:
        if self.error:
            msg = f"watchdog: communicator error during {self.phase} after step {step}: {self.error}"
        else:
            msg = (f"watchdog: no progress for {idle:.1f}s during {self.phase} after step {step} "
                   "(peer lost or collective hung)")
        path = os.environ.get("TFK_TERMINATION_LOG")
        if path:
            try:
                with open(path, "w") as f:
                    f.write(msg)
            except OSError:
                pass
        print(json.dumps({"event": "error", "kind": "comm_error" if self.error else "watchdog", "step": step,
                          "phase": self.phase, "idle_s": round(idle, 2), "message": msg,
                          "rccl_transport": _transport()}, sort_keys=True), flush=True)
        n = abort_communicators()
        print(json.dumps({"event": "comm_aborted", "communicators": n}, sort_keys=True), flush=True)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(self.exit_code)


def _comm_module():
    return sys.modules.get(__name__.rsplit(".", 2)[0] + ".parallel.tfk_comm")


def comm_async_error() -> str:
    """ncclCommGetAsyncError over every live tfk_comm communicator ("" = healthy)."""
    mod = _comm_module()
    return mod.async_errors() if mod is not None else ""


def _transport() -> dict:
    mod = sys.modules.get(__name__.rsplit(".", 2)[0] + ".parallel.comm")
    try:
        return mod.transport_summary() if mod is not None else {}
    except Exception:  # pragma: no cover
        return {}


def abort_communicators() -> int:
    """ncclCommAbort every live RCCL communicator of this process (parallel/tfk_comm). gloo groups
    of the CPU tier need no abort: os._exit closes their sockets and the peers' pending ops fail."""
    mod = _comm_module()
    if mod is None:  # never imported -> no communicator exists; do not pay a torch import here
        return 0
    try:
        return mod.abort_all()
    except Exception:  # pragma: no cover - the process is exiting anyway
        return 0
