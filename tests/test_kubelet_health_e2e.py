"""Node-level lifecycle goals of the reference through the native control plane (tfk-cluster:
apiserver + operator + gang scheduler + kubelet), CPU replicas:

* health checking (k8s-operator.md:1): a replica that wedges before training (here: the chief of
  restart generation 0 sleeps instead of starting the runtime) never touches its heartbeat file,
  its exec livenessProbe (runtime/health.py) fails, the kubelet kills it (exit 143, retryable) and
  the operator restarts the gang, which then trains to Succeeded; readinessProbe drives
  containerStatuses[].ready and the pod's Ready condition; tcpSocket / httpGet handlers.
* OOM (:5): resources.limits.memory is enforced on the container's resident set; a breach is
  SIGKILLed with reason OOMKilled, which is permanent -> the job fails with OOMKilled.
* storage (:2): a persistentVolumeClaim volume mounted at /tfk-ckpt in chief, worker
  and evaluator holds the checkpoints; after a retryable fault the gang resumes from the checkpoint
  on that volume, and the evaluator evaluates the final one from the same volume. An emptyDir
  holds the heartbeat file and disappears with its pod.
"""
import json
import os
import time

import pytest

from tensorflow_k8s_amd.control.client import LocalCluster, tfjob_condition

TRAIN = ["python3", "-m", "tensorflow_k8s_amd.runtime.train"]
HEALTH = "python3 -m tensorflow_k8s_amd.runtime.health --max-age 20 $TFK_HEARTBEAT_FILE"


def _events(text):
    return [json.loads(l) for l in text.splitlines() if l.startswith("{")]


def _wait(pred, timeout, what):
    dl = time.time() + timeout
    while time.time() < dl:
        v = pred()
        if v:
            return v
        time.sleep(0.2)
    raise AssertionError(f"timed out: {what}")


@pytest.fixture
def cluster(tmp_path, control_plane_bin, native_ext):
    with LocalCluster(root_dir=str(tmp_path / "cluster")) as c:
        yield c


def _container(cmd, args=(), env=(), **extra):
    c = {"name": "tensorflow", "image": "tfk/runtime", "command": cmd, "args": list(args),
         "env": [{"name": k, "value": v} for k, v in env]}
    c.update(extra)
    return c


def _job(name, specs, backoff=3):
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"tfReplicaSpecs": specs, "runPolicy": {"backoffLimit": backoff, "cleanPodPolicy": "None"}}}


def _rs(n, container, policy="ExitCode", volumes=()):
    return {"replicas": n, "restartPolicy": policy,
            "template": {"spec": {"containers": [container], "volumes": list(volumes),
                                  "terminationGracePeriodSeconds": 2}}}


def _cluster_events(c, reason):
    return [e for e in c.list("events") if e.get("reason") == reason]


def test_liveness_probe_kills_wedged_replica_and_gang_restarts(cluster):
    c = cluster.client
    args = ["--model", "lenet", "--steps", "8", "--batch", "16", "--device", "cpu", "--log-every", "4"]
    # generation 0 of the chief wedges before the runtime starts: no heartbeat is ever written
    wedge = ["sh", "-c", 'if [ "$TFK_RESTART_GENERATION" = "0" ]; then sleep 300; fi; exec "$@"', "sh"] + TRAIN
    probe = {"exec": {"command": ["sh", "-c", HEALTH]}, "initialDelaySeconds": 2, "periodSeconds": 1,
             "timeoutSeconds": 10, "failureThreshold": 3}
    hb = [{"name": "hb", "emptyDir": {}}]
    mounts = [{"name": "hb", "mountPath": "/tfk-hb"}]
    env = [("TFK_HEARTBEAT_FILE", "/tfk-hb/alive")]
    chief = _container(wedge, args, env, livenessProbe=probe, volumeMounts=mounts)
    worker = _container(TRAIN, args, env, livenessProbe=dict(probe, initialDelaySeconds=30), volumeMounts=mounts)
    c.create(_job("wedge", {"Chief": _rs(1, chief, volumes=hb), "Worker": _rs(1, worker, volumes=hb)}))
    j = c.wait_tfjob("wedge", timeout=240)
    st = j["status"]
    assert tfjob_condition(j) == "Succeeded", (st, c.logs("wedge-chief-0")[-2000:])
    assert st.get("restartCount") == 1 and any(cd["type"] == "Restarting" for cd in st["conditions"]), st
    unhealthy = [e for e in _cluster_events(c, "Unhealthy") if e["involvedObject"]["name"] == "wedge-chief-0"]
    assert unhealthy and "Liveness probe failed" in unhealthy[0]["message"], unhealthy
    ev = _events(c.logs("wedge-chief-0"))
    start = [e for e in ev if e.get("event") == "start"]
    assert start and start[-1]["restart_generation"] == 1, start
    assert [e for e in ev if e.get("event") == "done"][-1]["step"] == 8


def test_readiness_probe_drives_container_ready(cluster, tmp_path):
    c = cluster.client
    flag = str(tmp_path / "ready-flag")
    cmd = ["python3", "-c", f"import time, pathlib; time.sleep(2.5); pathlib.Path({flag!r}).touch(); time.sleep(6)"]
    ready = {"exec": {"command": ["test", "-f", flag]}, "periodSeconds": 0.3, "failureThreshold": 1}
    # a tcpSocket liveness probe against a closed port would kill it; against the apiserver it passes
    port = int(cluster.url.rsplit(":", 1)[1])
    live = {"tcpSocket": {"port": port}, "periodSeconds": 0.5}
    startup = {"httpGet": {"path": "/healthz", "port": port}, "periodSeconds": 0.3, "failureThreshold": 20}
    c.create(_job("ready", {"Chief": _rs(1, _container(cmd, readinessProbe=ready, livenessProbe=live,
                                                       startupProbe=startup))}))

    def status():
        try:
            p = c.get("pods", "ready-chief-0")
        except Exception:  # noqa: BLE001 -- not created yet
            return None
        cs = p.get("status", {}).get("containerStatuses") or []
        return (p["status"], cs[0]) if cs and "running" in cs[0].get("state", {}) else None
    st, cs = _wait(status, 60, "container running")
    assert cs["ready"] is False, cs  # not before the readiness probe succeeded
    st, cs = _wait(lambda: (lambda s: s if s and s[1]["ready"] else None)(status()), 30, "container ready")
    assert cs["started"] is True
    assert [cd["status"] for cd in st["conditions"] if cd["type"] == "Ready"] == ["True"], st
    j = c.wait_tfjob("ready", timeout=60)
    assert tfjob_condition(j) == "Succeeded", j["status"]
    assert not _cluster_events(c, "Unhealthy")


def test_memory_limit_breach_fails_job_oomkilled(cluster):
    c = cluster.client
    hog = ["python3", "-c", "import time\nb = bytearray(400 << 20)\nfor i in range(0, len(b), 4096): b[i] = 1\n"
           "time.sleep(60)"]
    ctr = _container(hog, resources={"limits": {"memory": "128Mi"}})
    c.create(_job("hog", {"Chief": _rs(1, ctr)}))
    j = c.wait_tfjob("hog", timeout=120)
    assert tfjob_condition(j) == "Failed", j["status"]
    msg = [cd for cd in j["status"]["conditions"] if cd["type"] == "Failed"][0]["message"]
    assert "OOMKilled" in msg, msg
    cs = c.get("pods", "hog-chief-0")["status"]["containerStatuses"][0]
    term = cs["state"]["terminated"]
    assert term["reason"] == "OOMKilled" and term["exitCode"] == 137, cs
    assert "memory limit exceeded" in term.get("message", ""), term
    assert j["status"].get("restartCount", 0) == 0  # permanent: no gang restart


@pytest.mark.parametrize("mode", ["auto", "substitute"])
def test_checkpoint_on_declared_volume_resume_and_evaluator(tmp_path, control_plane_bin, native_ext, mode):
    """Chief + worker + evaluator share a persistentVolumeClaim volume at /tfk-ckpt: the worker is
    SIGKILLed at step 10 in generation 0 (retryable) -> gang restart -> the chief restores step 8 from
    the volume; the evaluator (outside the training world) evaluates the final checkpoint there.
    auto: bind mounts in a private mount namespace where the kubelet may create one (root), else
    path substitution; substitute: forced path rewrite + TFK_VOLUME_MAP."""
    with LocalCluster(root_dir=str(tmp_path / "cluster"), extra_args=["--volume-mode", mode]) as cl:
        _volume_job(cl, tmp_path)
        log = open(cl.log_path).read()
    assert ("volume mounts" in log) == (mode == "auto")


def _volume_job(cluster, tmp_path):
    c = cluster.client
    ck = "/tfk-ckpt/run"
    args = ["--model", "lenet", "--steps", "16", "--batch", "16", "--device", "cpu", "--log-every", "4",
            "--checkpoint-dir", ck, "--checkpoint-every", "4"]
    fault = [("TFK_FAULT_AT_STEP", "10"), ("TFK_FAULT_EXIT", "137"), ("TFK_FAULT_RANK", "1")]
    vol = [{"name": "ckpt", "persistentVolumeClaim": {"claimName": "lenet-ckpt"}}]
    mnt = [{"name": "ckpt", "mountPath": "/tfk-ckpt"}]
    evaluator = _container(TRAIN, ["--model", "lenet", "--batch", "16", "--device", "cpu", "--checkpoint-dir", ck,
                                   "--eval-batches", "2", "--eval-timeout", "120"], volumeMounts=mnt)
    c.create(_job("vol", {"Chief": _rs(1, _container(TRAIN, args, fault, volumeMounts=mnt), volumes=vol),
                          "Worker": _rs(1, _container(TRAIN, args, fault, volumeMounts=mnt), volumes=vol),
                          "Evaluator": _rs(1, evaluator, policy="OnFailure", volumes=vol)}))
    j = c.wait_tfjob("vol", timeout=300)
    st = j["status"]
    assert tfjob_condition(j) == "Succeeded", (st, c.logs("vol-chief-0")[-2000:])
    assert st.get("restartCount") == 1, st
    ev = _events(c.logs("vol-chief-0"))
    restored = [e for e in ev if e.get("event") == "restored"]
    assert restored and restored[-1]["step"] == 8, [e for e in ev if e.get("event") != "train"]
    host = os.path.join(str(tmp_path), "cluster", "kubelet", "pvc", "default", "lenet-ckpt", "run")
    assert os.path.exists(os.path.join(host, "model.ckpt-16.index")), os.listdir(os.path.dirname(host))
    assert "model.ckpt-16" in open(os.path.join(host, "checkpoint")).read()
    assert not os.path.exists(ck)  # nothing was written at the mount path itself on the host
    evals = _wait(lambda: [e for e in _events(c.logs("vol-evaluator-0")) if e.get("event") == "eval"
                           and e["step"] == 16], 60, "evaluator eval of the final checkpoint")
    assert evals[-1]["loss"] == evals[-1]["loss"]


def test_bad_volume_blocks_container_with_failed_mount(cluster, tmp_path):
    """A hostPath volume of type Directory that does not exist: the container is never started
    (waiting, CreateContainerConfigError) and the kubelet records a FailedMount event; a readOnly
    mount of an existing directory is bind-mounted / substituted like any other."""
    c = cluster.client
    missing = str(tmp_path / "nope")
    ctr = _container(["python3", "-c", "pass"], volumeMounts=[{"name": "v", "mountPath": "/tfk-missing"}])
    c.create(_job("badvol", {"Chief": _rs(1, ctr, volumes=[{"name": "v", "hostPath": {"path": missing,
                                                                                       "type": "Directory"}}])}))

    def waiting():
        try:
            p = c.get("pods", "badvol-chief-0")
        except Exception:  # noqa: BLE001 -- not created yet
            return None
        cs = p.get("status", {}).get("containerStatuses") or []
        w = cs[0]["state"].get("waiting", {}) if cs else {}
        return w if w.get("reason") == "CreateContainerConfigError" else None
    _wait(waiting, 60, "CreateContainerConfigError")
    ev = _wait(lambda: _cluster_events(c, "FailedMount"), 30, "FailedMount event")
    assert missing in ev[0]["message"], ev
    assert not os.path.exists(missing)
