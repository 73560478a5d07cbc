"""Operator deployment paths a real cluster uses, end to end with the native binaries:

* HTTPS + bearer token: tfk-apiserver --tls-cert-file/--token-auth-file; tfk-operator configured
  only through a YAML kubeconfig (clusters/users/contexts, certificate-authority, token) --
  clientcmd.BuildConfigFromFlags in the reference (k8s-operator.md:92-101).
* HA failover: two tfk-operator --leader-elect replicas against one apiserver; SIGKILL the lease
  holder, the standby takes the Lease and reconciles a TFJob created afterwards
  (leaderelection, k8s-operator.md:59,237).
"""
import os
import signal
import subprocess
import time

import pytest

from tensorflow_k8s_amd.control.client import BIN, ApiError, TfkClient


def _job(name):
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"tfReplicaSpecs": {"Worker": {"replicas": 1, "restartPolicy": "Never", "template": {"spec": {
                "containers": [{"name": "tensorflow", "image": "tfk/runtime", "command": ["true"]}]}}}}}}


def _wait(pred, timeout, what):
    dl = time.time() + timeout
    while time.time() < dl:
        v = pred()
        if v:
            return v
        time.sleep(0.1)
    raise AssertionError(f"timed out waiting for {what}")


def _created(c, name):
    try:
        j = c.get("tfjobs", name)
    except ApiError:
        return False
    return any(cd["type"] == "Created" for cd in j.get("status", {}).get("conditions", []))


class Proc:
    def __init__(self, args, log):
        self.log = open(log, "w")
        self.p = subprocess.Popen(args, stdout=self.log, stderr=subprocess.STDOUT, start_new_session=True)

    def kill(self, sig=signal.SIGTERM):
        if self.p.poll() is None:
            os.killpg(self.p.pid, sig)
            try:
                self.p.wait(15)
            except subprocess.TimeoutExpired:
                os.killpg(self.p.pid, signal.SIGKILL)
                self.p.wait()
        self.log.close()


def _apiserver(tmp_path, extra=()):
    pf = tmp_path / "port"
    p = Proc([os.path.join(BIN, "tfk-apiserver"), "--port", "0", "--port-file", str(pf), *extra],
             str(tmp_path / "apiserver.log"))
    _wait(lambda: pf.exists() and pf.read_text().strip(), 30, "apiserver port")
    return p, int(pf.read_text())


@pytest.fixture
def tls_material(tmp_path):
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=tfk",
                    "-addext", "subjectAltName=IP:127.0.0.1,DNS:localhost", "-keyout", str(tmp_path / "tls.key"),
                    "-out", str(tmp_path / "tls.crt")], check=True, capture_output=True)
    (tmp_path / "tokens.csv").write_text("op-token,system:serviceaccount:kubeflow:tf-operator,1\n")
    return tmp_path


def test_operator_over_https_with_kubeconfig_token(tls_material, control_plane_bin):
    d = tls_material
    api, port = _apiserver(d, ["--tls-cert-file", str(d / "tls.crt"), "--tls-private-key-file", str(d / "tls.key"),
                               "--token-auth-file", str(d / "tokens.csv")])
    url = f"https://127.0.0.1:{port}"
    (d / "kubeconfig").write_text(f"""apiVersion: v1
kind: Config
current-context: tfk
clusters:
- name: local
  cluster:
    server: {url}
    certificate-authority: tls.crt
contexts:
- name: tfk
  context:
    cluster: local
    user: operator
    namespace: default
users:
- name: operator
  user:
    token: op-token
""")
    op = Proc([os.path.join(BIN, "tfk-operator"), "--kubeconfig", str(d / "kubeconfig"), "--leader-elect=false",
               "--resync-period", "2", "--gang-scheduling=false"], str(d / "operator.log"))
    try:
        anon = TfkClient(url, ca=str(d / "tls.crt"))
        with pytest.raises(ApiError) as e:
            anon.list("tfjobs")
        assert e.value.code == 401
        c = TfkClient(url, token="op-token", ca=str(d / "tls.crt"))
        c.create(_job("secure"))
        _wait(lambda: _created(c, "secure"), 30, "Created condition over https")
        pods = _wait(lambda: c.list("pods", label_selector="tf-job-name=secure"), 30, "pods")
        assert pods
        assert op.p.poll() is None, open(d / "operator.log").read()[-2000:]
        log = open(d / "operator.log").read()
        assert "bearer-token" in log and url in log
    finally:
        op.kill()
        api.kill()


def test_leader_failover_two_operators(tmp_path, control_plane_bin):
    api, port = _apiserver(tmp_path)
    url = f"http://127.0.0.1:{port}"
    c = TfkClient(url)
    common = ["--apiserver", url, "--leader-elect", "--lease-duration", "2", "--renew-deadline", "1.5",
              "--retry-period", "0.25", "--resync-period", "2", "--gang-scheduling=false"]
    ops = {i: Proc([os.path.join(BIN, "tfk-operator"), *common, "--identity", i], str(tmp_path / f"op-{i}.log"))
           for i in ("op-a", "op-b")}
    try:
        def holder():
            try:
                return c.get("leases", "tf-operator")["spec"].get("holderIdentity")
            except ApiError:
                return None
        first = _wait(holder, 30, "first leader")
        c.create(_job("before"))
        _wait(lambda: _created(c, "before"), 30, "job reconciled by the first leader")
        ops[first].kill(signal.SIGKILL)  # no graceful lease release
        standby = "op-b" if first == "op-a" else "op-a"
        _wait(lambda: holder() == standby, 30, "standby takes the lease")
        c.create(_job("after"))
        _wait(lambda: _created(c, "after"), 30, "job reconciled by the new leader")
        assert ops[standby].p.poll() is None
        log = open(tmp_path / f"op-{standby}.log").read()
        assert "after" in log or _created(c, "after")
    finally:
        for p in ops.values():
            p.kill()
        api.kill()
