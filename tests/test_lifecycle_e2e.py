"""TFJob lifecycle branches driven end to end through tfk-cluster (apiserver + operator + gang
scheduler + kubelet) with trivial containers: run policy (ttlSecondsAfterFinished,
activeDeadlineSeconds, cleanPodPolicy All / Running / None) and a reference-era v1alpha1 job
(replicaSpecs list, MASTER chief) driven to phase Done. Reference: full lifecycle management
(k8s-operator.md:1), run-to-completion Job semantics and kept completed pods (:44-52).
"""
import time

import pytest

from tensorflow_k8s_amd.control.client import ApiError, LocalCluster, tfjob_condition

SLEEP = ["python3", "-c", "import time; time.sleep(120)"]
OK = ["python3", "-c", "pass"]


def _rs(n, cmd, policy="Never"):
    return {"replicas": n, "restartPolicy": policy, "template": {"spec": {"containers": [{
        "name": "tensorflow", "image": "tfk/runtime", "command": cmd}]}}}


def _job(name, specs, **run_policy):
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"tfReplicaSpecs": specs, "runPolicy": run_policy}}


def _wait(pred, timeout, what):
    dl = time.time() + timeout
    while time.time() < dl:
        v = pred()
        if v:
            return v
        time.sleep(0.2)
    raise AssertionError(f"timed out: {what}")


def _pod_names(c, job):
    return sorted(p["metadata"]["name"] for p in c.list("pods", label_selector=f"tf-job-name={job}")
                  if not p["metadata"].get("deletionTimestamp"))


@pytest.fixture
def cluster(tmp_path, control_plane_bin):
    with LocalCluster(root_dir=str(tmp_path / "cluster")) as c:
        yield c


def test_ttl_seconds_after_finished_deletes_job(cluster):
    c = cluster.client
    c.create(_job("ttl", {"Chief": _rs(1, OK)}, ttlSecondsAfterFinished=1, cleanPodPolicy="None"))
    j = c.wait_tfjob("ttl", timeout=60)
    assert tfjob_condition(j) == "Succeeded"

    def gone():
        try:
            c.get("tfjobs", "ttl")
            return False
        except ApiError as e:
            return e.code == 404
    _wait(gone, 30, "TTL deletion")
    # owner-reference GC takes the pods and services with it
    _wait(lambda: not _pod_names(c, "ttl"), 30, "pods garbage-collected")


def test_active_deadline_fails_and_stops_pods(cluster):
    c = cluster.client
    c.create(_job("deadline", {"Chief": _rs(1, SLEEP), "Worker": _rs(1, SLEEP)}, activeDeadlineSeconds=2,
                  cleanPodPolicy="None"))
    j = c.wait_tfjob("deadline", timeout=60)
    assert tfjob_condition(j) == "Failed"
    failed = [cd for cd in j["status"]["conditions"] if cd["type"] == "Failed"][0]
    assert failed["reason"] == "DeadlineExceeded", failed
    # running replicas are stopped even with cleanPodPolicy None (the job is over)
    _wait(lambda: all(p["status"].get("phase") in ("Failed", "Succeeded")
                      for p in c.list("pods", label_selector="tf-job-name=deadline")) or not _pod_names(c, "deadline"),
          30, "deadline pods stopped")


@pytest.mark.parametrize("policy,expect_left", [("All", []), ("Running", ["cp-running-chief-0"]),
                                                ("None", ["cp-none-chief-0", "cp-none-worker-0"])])
def test_clean_pod_policy(cluster, policy, expect_left):
    """Chief finishes (job Succeeded) while the worker still runs: All deletes every pod, Running
    deletes the still-running worker only, None keeps both (k8s-operator.md:51: completed pods are
    not auto-deleted)."""
    c = cluster.client
    name = f"cp-{policy.lower()}"
    c.create(_job(name, {"Chief": _rs(1, OK), "Worker": _rs(1, SLEEP)}, cleanPodPolicy=policy))
    j = c.wait_tfjob(name, timeout=60)
    assert tfjob_condition(j) == "Succeeded", j["status"]
    _wait(lambda: _pod_names(c, name) == expect_left, 30, f"cleanPodPolicy {policy} -> {expect_left}")
    time.sleep(1.0)
    assert _pod_names(c, name) == expect_left
    if policy == "None":
        c.delete("pods", f"{name}-worker-0")


def test_v1alpha1_job_runs_to_done(cluster):
    """Reference-era TFJob (tensorflow/k8s v1alpha1: replicaSpecs list, tfReplicaType, MASTER chief,
    runtimeId, phase/state status) served through the v1 hub and driven to phase Done."""
    c = cluster.client
    c.create({"apiVersion": "kubeflow.org/v1alpha1", "kind": "TFJob",
              "metadata": {"name": "legacy", "namespace": "default"},
              "spec": {"replicaSpecs": [
                  {"replicas": 1, "tfReplicaType": "MASTER", "template": {"spec": {"restartPolicy": "OnFailure",
                   "containers": [{"name": "tensorflow", "image": "tfk/runtime", "command": OK}]}}},
                  {"replicas": 1, "tfReplicaType": "WORKER", "template": {"spec": {"restartPolicy": "OnFailure",
                   "containers": [{"name": "tensorflow", "image": "tfk/runtime", "command": OK}]}}}]}})

    def done():
        j = c.get("tfjobs", "legacy", version="v1alpha1")
        return j if j.get("status", {}).get("phase") == "Done" else None
    j = _wait(done, 60, "v1alpha1 phase Done")
    assert j["status"]["state"] == "Succeeded", j["status"]
    assert j["status"]["replicaStatuses"], j["status"]
    # the same object through the v1 hub
    v1 = c.get("tfjobs", "legacy", version="v1")
    assert tfjob_condition(v1) == "Succeeded"
