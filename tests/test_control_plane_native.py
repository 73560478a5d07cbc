"""Native control-plane unit tests (cpp/main/unit-tests.cc: API defaults/validation/conversion,
TF_CONFIG, apiserver store semantics, informer, workqueue, leader election, gang placement,
trainer reconcile incl. gang restart / permanent failure / OOM / finalizer cleanup, TF bundle),
plus the same binary under ThreadSanitizer and AddressSanitizer."""
import os
import subprocess

import pytest

from conftest import ROOT


def _run(binary, env=None):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=600, env={**os.environ, **(env or {})})
    return r.returncode, r.stdout, r.stderr


def test_unit_tests(control_plane_bin):
    rc, out, err = _run(os.path.join(control_plane_bin, "tfk-unit-tests"))
    assert rc == 0, out[-3000:] + err[-2000:]
    assert " 0 failed" in out


@pytest.mark.parametrize("san", ["thread", "address"])
def test_unit_tests_sanitized(san):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "cpp"), f"-j{max(2, min(8, os.cpu_count() or 2) // 2)}", f"SAN={san}"],
                       capture_output=True, text=True, timeout=1800)
    assert r.returncode == 0, r.stderr[-3000:]
    env = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1", "ASAN_OPTIONS": "detect_leaks=1"}
    rc, out, err = _run(os.path.join(ROOT, "build", f"bin-{san}", "tfk-unit-tests"), env)
    assert rc == 0, out[-2000:] + err[-4000:]
    assert "ThreadSanitizer" not in err and "AddressSanitizer" not in err, err[-4000:]
