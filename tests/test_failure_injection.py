"""Failure modes named by the reference (k8s-operator.md:5: OOM, port already in use, disk
failure), injected at the runtime boundary (the operator-side handling is in test_operator_e2e.py).

Port in use: the chief's rendezvous port (tfPort, TF_CONFIG) is held by another process -- in
practice the previous restart generation still shutting down. init_process_group retries, then
raises RendezvousError, and the replica exits 143 (retryable: the operator restarts the gang)
with the reason in its termination log.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from tensorflow_k8s_amd.parallel import cluster

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _held_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(1)
    return s, s.getsockname()[1]


def test_rendezvous_port_in_use_raises_retryable():
    s, port = _held_port()
    try:
        info = cluster.ClusterInfo(task_type="chief", task_index=0, rank=0, world_size=2, master_addr="127.0.0.1",
                                   master_port=port, worker_ranks=[0, 1], source="tf_config")
        with pytest.raises(cluster.RendezvousError) as e:
            cluster.init_process_group(info, "gloo", timeout_s=5, retries=2)
        assert "port already in use" in str(e.value)
        assert cluster.RendezvousError.exit_code == 143
    finally:
        s.close()


def test_chief_replica_exits_143_on_port_in_use(tmp_path):
    s, port = _held_port()
    try:
        tf = {"cluster": {"chief": [f"127.0.0.1:{port}"], "worker": ["127.0.0.1:1"]},
              "task": {"type": "chief", "index": 0}, "environment": "cloud"}
        env = dict(os.environ, TF_CONFIG=json.dumps(tf), TFK_TERMINATION_LOG=str(tmp_path / "term"),
                   PYTHONPATH=ROOT, TFK_RENDEZVOUS_RETRIES="1")
        r = subprocess.run([sys.executable, "-m", "tensorflow_k8s_amd.runtime.train", "--model", "lenet", "--steps", "2",
                            "--device", "cpu", "--rendezvous-timeout", "5"], env=env, capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 143, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
        assert "port already in use" in (tmp_path / "term").read_text()
        ev = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        assert ev[-1]["kind"] == "rendezvous"
    finally:
        s.close()


def test_nonfinite_loss_fails_permanently(tmp_path):
    """Silent numeric corruption (TFK_FAULT_EXIT=nan poisons the weights after step 2): the replica
    stops at the next metrics point with exit 1 (permanent: a restart would replay the same state)
    and a NonFiniteLoss termination reason, before the corrupt weights reach a checkpoint."""
    env = dict(os.environ, TFK_TERMINATION_LOG=str(tmp_path / "term"), PYTHONPATH=ROOT, TFK_FAULT_AT_STEP="2",
               TFK_FAULT_EXIT="nan")
    env.pop("TF_CONFIG", None)
    r = subprocess.run([sys.executable, "-m", "tensorflow_k8s_amd.runtime.train", "--model", "lenet", "--steps", "8",
                        "--device", "cpu", "--log-every", "4", "--checkpoint-dir", str(tmp_path / "ckpt"),
                        "--checkpoint-every", "4"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 1, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "NonFiniteLoss" in (tmp_path / "term").read_text()
    ev = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert ev[-1]["kind"] == "numerics"
    assert not [e for e in ev if e.get("event") == "checkpoint" and e.get("step", 0) >= 4]


def test_sigterm_flushes_inflight_checkpoint(tmp_path):
    """A graceful stop (the kubelet's SIGTERM on gang restart / resize) while an asynchronous
    checkpoint write is in flight: the replica lets the write finish, then exits 143 -- the next
    generation resumes from that checkpoint instead of an older one (or none)."""
    import signal
    import time
    env = dict(os.environ, PYTHONPATH=ROOT, TFK_FAULT_CKPT_DELAY_S="2")
    env.pop("TF_CONFIG", None)
    ck = tmp_path / "ck"
    p = subprocess.Popen([sys.executable, "-u", "-m", "tensorflow_k8s_amd.runtime.train", "--model", "lenet",
                          "--steps", "1000", "--device", "cpu", "--checkpoint-dir", str(ck), "--checkpoint-every", "3",
                          "--step-sleep", "0.05"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    lines = []
    try:
        dl = time.time() + 120
        while time.time() < dl:
            line = p.stdout.readline()
            if not line:
                break
            lines.append(line)
            if '"event": "checkpoint"' in line:
                p.send_signal(signal.SIGTERM)  # the write stalls 2 s: it is in flight now
                break
        out, _ = p.communicate(timeout=60)
        lines.append(out)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 143, "".join(lines)[-2000:]
    ev = [json.loads(l) for l in "".join(lines).splitlines() if l.startswith("{")]
    term = [e for e in ev if e.get("event") == "terminated"]
    assert term and term[-1]["checkpoint_flushed"] is True, ev[-3:]
    assert (ck / "model.ckpt-3.index").exists() and "model.ckpt-3" in (ck / "checkpoint").read_text()
