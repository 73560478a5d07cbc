"""Tracing for the in-pod runtime: roctx ranges + a Chrome-trace step timeline.

* ``roctx`` ranges (``libroctx64.so`` via ctypes) wrap every traced span, so a
  ``rocprofv3 --marker-trace`` run shows forward/backward/all-reduce/optimizer/checkpoint phases
  around the HIP kernels they launch. Absent library -> ranges are no-ops.
* Host timeline: each span records wall-clock begin/end (and, with ``device_events=True``, a
  pair of HIP events so the device time of the span is known after a sync). ``dump(path)``
  writes Chrome trace-event JSON (chrome://tracing, Perfetto) with one track per rank.

Usage::

    tr = Tracer(rank=0)
    with tr.span("step", step=3):
        ...
    tr.dump("trace_rank0.json")
"""
from __future__ import annotations

import ctypes
import ctypes.util
import json
import os
import threading
import time
from contextlib import contextmanager

_ROCTX = None
_ROCTX_TRIED = False


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if not _ROCTX_TRIED:
        _ROCTX_TRIED = True
        cands = [os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "libroctx64.so"),
                 ctypes.util.find_library("roctx64") or ""]
        for c in cands:
            if c and os.path.exists(c):
                try:
                    lib = ctypes.CDLL(c)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    _ROCTX = lib
                    break
                except OSError:
                    continue
    return _ROCTX


def roctx_available() -> bool:
    return _roctx() is not None


class Tracer:
    def __init__(self, rank: int = 0, enabled: bool = True, device_events: bool = False, max_events: int = 200_000):
        self.rank, self.enabled, self.device_events = rank, enabled, device_events
        self.max_events = max_events
        self.events: list[dict] = []
        self._pending = []  # (event dict, start hip event, end hip event)
        self._t0 = time.perf_counter()
        self._lock = threading.Lock()
        self._use_roctx = enabled and roctx_available()

    def _now_us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    @contextmanager
    def span(self, name: str, cat: str = "runtime", **args):
        if not self.enabled:
            yield
            return
        if self._use_roctx:
            _ROCTX.roctxRangePushA(name.encode())
        ev0 = ev1 = None
        if self.device_events:
            import torch
            if torch.cuda.is_available():
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
        t0 = self._now_us()
        try:
            yield
        finally:
            t1 = self._now_us()
            if ev1 is not None:
                ev1.record()
            if self._use_roctx:
                _ROCTX.roctxRangePop()
            e = {"name": name, "cat": cat, "ph": "X", "ts": round(t0, 3), "dur": round(t1 - t0, 3),
                 "pid": self.rank, "tid": threading.get_ident() % 100000, "args": dict(args)}
            with self._lock:
                if len(self.events) < self.max_events:
                    self.events.append(e)
                    if ev0 is not None:
                        self._pending.append((e, ev0, ev1))

    def instant(self, name: str, cat: str = "runtime", **args) -> None:
        if not self.enabled:
            return
        with self._lock:
            if len(self.events) < self.max_events:
                self.events.append({"name": name, "cat": cat, "ph": "i", "s": "p", "ts": round(self._now_us(), 3),
                                    "pid": self.rank, "tid": threading.get_ident() % 100000, "args": dict(args)})

    def resolve_device_times(self) -> None:
        """Synchronize and attach the device duration (ms) of every span that recorded events."""
        if not self._pending:
            return
        import torch
        torch.cuda.synchronize()
        with self._lock:
            for e, a, b in self._pending:
                e["args"]["device_ms"] = round(a.elapsed_time(b), 4)
            self._pending = []

    def to_chrome(self) -> dict:
        self.resolve_device_times()
        meta = [{"name": "process_name", "ph": "M", "pid": self.rank, "args": {"name": f"rank {self.rank}"}}]
        return {"traceEvents": meta + list(self.events), "displayTimeUnit": "ms"}

    def dump(self, path: str) -> str:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(self.to_chrome(), f)
        os.replace(tmp, path)
        return path


NULL_TRACER = Tracer(enabled=False)
