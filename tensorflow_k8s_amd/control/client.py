"""Python REST client for tfk-apiserver (the kubectl-side of the control plane) and helpers to
launch the native control-plane binaries built from cpp/ (tfk-cluster, tfk-operator, ...)."""
from __future__ import annotations

import json
import os
import subprocess
import time
from typing import Any

import requests

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "build", "bin")

CORE = {"pods", "services", "events", "configmaps", "endpoints", "nodes", "namespaces"}
GROUPS = {"tfjobs": "kubeflow.org", "leases": "coordination.k8s.io", "podgroups": "scheduling.tfk.io",
          "customresourcedefinitions": "apiextensions.k8s.io", "priorityclasses": "scheduling.k8s.io"}
ALIASES = {"tfjob": "tfjobs", "tfj": "tfjobs", "pod": "pods", "po": "pods", "svc": "services", "service": "services",
           "event": "events", "ev": "events", "node": "nodes", "no": "nodes", "lease": "leases", "pg": "podgroups",
           "podgroup": "podgroups", "crd": "customresourcedefinitions", "ns": "namespaces", "pc": "priorityclasses",
           "priorityclass": "priorityclasses"}
KIND_PLURAL = {"TFJob": "tfjobs", "Pod": "pods", "Service": "services", "Event": "events", "Node": "nodes",
               "ConfigMap": "configmaps", "Lease": "leases", "PodGroup": "podgroups", "PriorityClass": "priorityclasses",
               "CustomResourceDefinition": "customresourcedefinitions", "Namespace": "namespaces"}


class ApiError(RuntimeError):
    def __init__(self, code: int, body: Any):
        self.code = code
        self.body = body
        msg = body.get("message") if isinstance(body, dict) else body
        super().__init__(f"HTTP {code}: {msg}")


class TfkClient:
    def __init__(self, server: str | None = None, tfjob_version: str = "v1", timeout: float = 30.0,
                 token: str | None = None, ca: str | None = None):
        """token: bearer token (tfk-apiserver --token-auth-file / a service account); ca: PEM bundle
        that signs an https:// server's certificate."""
        self.server = (server or os.environ.get("TFK_APISERVER", "http://127.0.0.1:8080")).rstrip("/")
        self.tfjob_version = tfjob_version
        self.timeout = timeout
        self.s = requests.Session()
        token = token or os.environ.get("TFK_TOKEN")
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.ca = ca

    def path(self, plural: str, ns: str | None = None, name: str | None = None, sub: str | None = None,
             version: str | None = None) -> str:
        plural = ALIASES.get(plural, plural)
        if plural in CORE:
            p = "/api/v1"
        else:
            g = GROUPS.get(plural)
            if g is None:
                raise ValueError(f"unknown resource {plural}")
            v = version or (self.tfjob_version if plural == "tfjobs" else ("v1beta1" if g == "apiextensions.k8s.io" else "v1"))
            p = f"/apis/{g}/{v}"
        if ns and plural not in ("nodes", "namespaces", "customresourcedefinitions", "priorityclasses"):
            p += f"/namespaces/{ns}"
        p += f"/{plural}"
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return self.server + p

    def _do(self, method, url, body=None, params=None, raw=False):
        r = self.s.request(method, url, data=json.dumps(body) if body is not None else None, params=params,
                           timeout=self.timeout, headers={"Content-Type": "application/json"},
                           **({"verify": self.ca} if self.ca else {}))  # explicit: REQUESTS_CA_BUNDLE would win
        if raw:
            if r.status_code >= 300:
                raise ApiError(r.status_code, r.text)
            return r.text
        try:
            j = r.json()
        except ValueError:
            j = r.text
        if r.status_code >= 300:
            raise ApiError(r.status_code, j)
        return j

    def create(self, obj: dict, ns: str | None = None) -> dict:
        plural = KIND_PLURAL[obj["kind"]]
        ns = ns or obj.get("metadata", {}).get("namespace", "default")
        ver = obj.get("apiVersion", "").split("/")[-1] if plural == "tfjobs" else None
        return self._do("POST", self.path(plural, ns, version=ver), obj)

    def apply(self, obj: dict, ns: str | None = None) -> dict:
        plural = KIND_PLURAL[obj["kind"]]
        ns = ns or obj.get("metadata", {}).get("namespace", "default")
        try:
            return self.create(obj, ns)
        except ApiError as e:
            if e.code != 409:
                raise
            ver = obj.get("apiVersion", "").split("/")[-1] if plural == "tfjobs" else None
            cur = self.get(plural, obj["metadata"]["name"], ns, version=ver)
            obj = dict(obj)
            obj["metadata"] = dict(obj.get("metadata", {}))
            obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
            return self._do("PUT", self.path(plural, ns, obj["metadata"]["name"], version=ver), obj)

    def get(self, plural: str, name: str, ns: str = "default", version: str | None = None) -> dict:
        return self._do("GET", self.path(plural, ns, name, version=version))

    def list(self, plural: str, ns: str | None = "default", label_selector: str = "", field_selector: str = "",
             version: str | None = None) -> list:
        params = {}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        return self._do("GET", self.path(plural, ns, version=version), params=params)["items"]

    def update(self, obj: dict, status: bool = False) -> dict:
        plural = KIND_PLURAL[obj["kind"]]
        md = obj["metadata"]
        return self._do("PUT", self.path(plural, md.get("namespace", "default"), md["name"], "status" if status else None), obj)

    def patch(self, plural: str, name: str, patch: dict, ns: str = "default") -> dict:
        return self._do("PATCH", self.path(plural, ns, name), patch)

    def delete(self, plural: str, name: str, ns: str = "default", propagation: str = "Background") -> dict:
        return self._do("DELETE", self.path(plural, ns, name), params={"propagationPolicy": propagation})

    def logs(self, pod: str, ns: str = "default", tail: int | None = None) -> str:
        return self._do("GET", self.path("pods", ns, pod, "log"), params={"tailLines": tail} if tail else None, raw=True)

    def healthy(self) -> bool:
        try:
            return self.s.get(self.server + "/healthz", timeout=2,
                              **({"verify": self.ca} if self.ca else {})).status_code == 200
        except requests.RequestException:
            return False

    def wait_tfjob(self, name: str, ns: str = "default", conditions=("Succeeded", "Failed"), timeout: float = 300,
                   poll: float = 0.2) -> dict:
        dl = time.time() + timeout
        while time.time() < dl:
            j = self.get("tfjobs", name, ns)
            st = j.get("status", {})
            for c in st.get("conditions", []):
                if c["type"] in conditions and c["status"] == "True":
                    return j
            if st.get("phase") in ("Done", "Failed") and any(s in conditions for s in ("Succeeded", "Failed")):
                return j
            time.sleep(poll)
        raise TimeoutError(f"tfjob {ns}/{name} did not reach {conditions} in {timeout}s: {j.get('status')}")


def tfjob_condition(job: dict) -> str | None:
    """Latest true condition type (v1) or state (v1alpha1)."""
    st = job.get("status", {})
    true = [c["type"] for c in st.get("conditions", []) if c.get("status") == "True"]
    for t in ("Succeeded", "Failed", "Restarting", "Running", "Created"):
        if t in true:
            return t
    return st.get("state")


class LocalCluster:
    """Spawns the native all-in-one control plane (apiserver + operator + gang scheduler + kubelet)."""

    def __init__(self, gpus: int = 0, root_dir: str | None = None, extra_args: list | None = None, env=None,
                 log_path: str | None = None):
        import tempfile
        self.root = root_dir or tempfile.mkdtemp(prefix="tfk-cluster-")
        os.makedirs(self.root, exist_ok=True)
        self.port_file = os.path.join(self.root, "port")
        self.log_path = log_path or os.path.join(self.root, "cluster.log")
        args = [os.path.join(BIN, "tfk-cluster"), "--port", "0", "--port-file", self.port_file, "--gpus", str(gpus),
                "--root-dir", os.path.join(self.root, "kubelet"), "--resync-period", "5"] + (extra_args or [])
        self.log = open(self.log_path, "w")
        e = dict(os.environ)
        e.update(env or {})
        e.setdefault("PYTHONPATH", ROOT)
        self.proc = subprocess.Popen(args, stdout=self.log, stderr=subprocess.STDOUT, env=e, start_new_session=True)
        dl = time.time() + 30
        port = None
        while time.time() < dl and port is None:
            if self.proc.poll() is not None:
                raise RuntimeError(f"tfk-cluster exited: {open(self.log_path).read()[-2000:]}")
            try:  # the binary renames a complete file into place; tolerate older binaries' partial writes
                port = int(open(self.port_file).read().strip())
            except (OSError, ValueError):
                time.sleep(0.05)
        if port is None:
            raise RuntimeError(f"tfk-cluster wrote no port within 30 s: {open(self.log_path).read()[-2000:]}")
        self.url = f"http://127.0.0.1:{port}"
        self.client = TfkClient(self.url)
        while not self.client.healthy():
            time.sleep(0.05)

    def stop(self):
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(15)
            except subprocess.TimeoutExpired:
                os.killpg(self.proc.pid, 9)
                self.proc.wait()
        self.log.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()
