"""Liveness heartbeat of a training replica, for the kubelet's probes (cpp/kubelet/probe.h).

The runtime touches ``$TFK_HEARTBEAT_FILE`` (when set) at every setup phase and training step, and
``python -m tensorflow_k8s_amd.runtime.health FILE --max-age S`` -- the exec handler of a pod's
livenessProbe -- exits 0 only while the file is younger than S seconds. A replica that wedges
before its in-process watchdog starts (import, rendezvous, a GIL-holding native call) stops
touching the file, its probe fails, and the kubelet kills it: exit 143 is retryable, so the
operator restarts the gang (k8s-operator.md:1 "health checking", :5 failure modes).

This module imports nothing heavy: the probe command runs every period.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

_path = os.environ.get("TFK_HEARTBEAT_FILE", "")
_last = 0.0
MIN_INTERVAL_S = 0.5  # touches are rate-limited (a step loop may run thousands of steps per second)


def beat(force: bool = False) -> None:
    """Touch the heartbeat file (no-op without TFK_HEARTBEAT_FILE)."""
    global _last
    if not _path:
        return
    now = time.monotonic()
    if not force and now - _last < MIN_INTERVAL_S:
        return
    _last = now
    try:
        with open(_path, "a"):
            pass
        os.utime(_path, None)
    except OSError:
        pass  # a full or read-only disk must not kill training; the probe will say so


def age_s(path: str) -> float:
    """Seconds since the heartbeat file was touched (inf if missing)."""
    try:
        return max(0.0, time.time() - os.stat(path).st_mtime)
    except OSError:
        return float("inf")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="exit 0 while the heartbeat file is fresh")
    ap.add_argument("file", nargs="?", default=_path)
    ap.add_argument("--max-age", type=float, default=60.0)
    a = ap.parse_args(argv)
    if not a.file:
        print("no heartbeat file (argument or TFK_HEARTBEAT_FILE)", file=sys.stderr)
        return 2
    age = age_s(a.file)
    if age <= a.max_age:
        return 0
    print(f"heartbeat {a.file} is {age:.1f} s old (max {a.max_age:g} s)", file=sys.stderr)
    return 1


if __name__ == "__main__":
    sys.exit(main())
