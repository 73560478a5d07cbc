"""End-to-end: native control plane (tfk-cluster: apiserver + TFJob operator + gang scheduler +
kubelet, cpp/) running real training replicas (runtime/train.py) on CPU.

Covers SURVEY §4.2 T3/T4: TFJob -> pods/services with TF_CONFIG -> MWMS training -> Succeeded;
retryable failure (exit 137) -> gang restart -> resume from the chief's checkpoint -> Succeeded
with the same final loss as an uninterrupted run; permanent failure (exit 1) -> Failed;
backoffLimit exhaustion -> Failed.
"""
import json
import os

import pytest

from tensorflow_k8s_amd.control.client import LocalCluster, tfjob_condition

TRAIN = ["python3", "-m", "tensorflow_k8s_amd.runtime.train"]


def _rs(n, args, env=(), policy="ExitCode"):
    return {"replicas": n, "restartPolicy": policy, "template": {"spec": {"containers": [{
        "name": "tensorflow", "image": "tfk/runtime", "command": TRAIN, "args": args,
        "env": [{"name": k, "value": v} for k, v in env]}]}}}


def _job(name, specs, backoff=3):
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"tfReplicaSpecs": specs, "runPolicy": {"backoffLimit": backoff, "cleanPodPolicy": "None"}}}


def _events(text):
    return [json.loads(l) for l in text.splitlines() if l.startswith("{")]


@pytest.fixture
def cluster(tmp_path, control_plane_bin, native_ext):
    with LocalCluster(root_dir=str(tmp_path / "cluster")) as c:
        yield c


def _args(ck, steps=16):
    return ["--model", "lenet", "--steps", str(steps), "--batch", "16", "--device", "cpu", "--log-every", "4",
            "--checkpoint-dir", ck, "--checkpoint-every", "4"]


def test_mnist_job_gang_restart_resumes_exactly(cluster, tmp_path):
    c = cluster.client
    # uninterrupted reference run
    ck0 = str(tmp_path / "ck0")
    c.create(_job("ref", {"Chief": _rs(1, _args(ck0)), "Worker": _rs(1, _args(ck0))}))
    j = c.wait_tfjob("ref", timeout=240)
    assert tfjob_condition(j) == "Succeeded", j["status"]
    ref_loss = [e for e in _events(c.logs("ref-chief-0")) if e["event"] == "done"][-1]["loss"]
    # worker 0 is SIGKILLed at step 10 in restart generation 0 -> retryable -> gang restart
    ck1 = str(tmp_path / "ck1")
    fault = [("TFK_FAULT_AT_STEP", "10"), ("TFK_FAULT_EXIT", "137"), ("TFK_FAULT_RANK", "1")]
    c.create(_job("flaky", {"Chief": _rs(1, _args(ck1), fault), "Worker": _rs(1, _args(ck1), fault)}))
    j = c.wait_tfjob("flaky", timeout=240)
    st = j["status"]
    assert tfjob_condition(j) == "Succeeded", st
    assert any(cd["type"] == "Restarting" for cd in st["conditions"]), st
    ev = _events(c.logs("flaky-chief-0"))
    restored = [e for e in ev if e["event"] == "restored"]
    assert restored and restored[-1]["step"] == 8
    loss = [e for e in ev if e["event"] == "done"][-1]["loss"]
    assert abs(loss - ref_loss) <= 1e-6 * max(1.0, abs(ref_loss)), (loss, ref_loss)
    # every replica got a TF_CONFIG with both roles and its own task
    pod = c.get("pods", "flaky-worker-0")
    env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0]["env"]}
    tf = json.loads(env["TF_CONFIG"])
    assert tf["task"] == {"type": "worker", "index": 0} and len(tf["cluster"]["chief"]) == 1


def test_permanent_failure_fails_job(cluster, tmp_path):
    c = cluster.client
    fault = [("TFK_FAULT_AT_STEP", "2"), ("TFK_FAULT_EXIT", "1"), ("TFK_FAULT_RANK", "0")]
    c.create(_job("bad", {"Chief": _rs(1, _args(str(tmp_path / "ck")), fault)}))
    j = c.wait_tfjob("bad", timeout=180)
    assert tfjob_condition(j) == "Failed", j["status"]


def test_backoff_limit_exhausted(cluster, tmp_path):
    c = cluster.client
    fault = [("TFK_FAULT_AT_STEP", "1"), ("TFK_FAULT_EXIT", "137"), ("TFK_FAULT_RANK", "0"),
             ("TFK_FAULT_GENERATION", "any")]
    c.create(_job("crashloop", {"Chief": _rs(1, _args(str(tmp_path / "ck")), fault)}, backoff=2))
    j = c.wait_tfjob("crashloop", timeout=240)
    assert tfjob_condition(j) == "Failed", j["status"]
    msg = [cd for cd in j["status"]["conditions"] if cd["type"] == "Failed"][0]["message"]
    assert "backoff" in msg.lower(), msg


def test_deploy_examples_are_accepted(cluster):
    """Every manifest under deploy/ is accepted by the apiserver (CRD schema, v1alpha1 conversion)
    and picked up by the operator (Created condition); GPU jobs stay Pending on this GPU-less node."""
    import glob

    import yaml
    c = cluster.client
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = []
    for f in sorted(glob.glob(os.path.join(root, "deploy", "examples", "*.yaml"))):
        obj = yaml.safe_load(open(f))
        c.create(obj)
        names.append(obj["metadata"]["name"])
    import time
    deadline = time.time() + 120  # generous: under pytest -n 4 the sanitizer builds load every core
    pending = set(names)
    while pending and time.time() < deadline:
        for n in list(pending):
            j = c.get("tfjobs", n)
            conds = j.get("status", {}).get("conditions", [])
            if any(cd["type"] == "Created" for cd in conds) or j.get("status", {}).get("phase"):
                pending.discard(n)
        time.sleep(0.2)
    for n in names:
        c.delete("tfjobs", n)
    assert not pending, pending


def test_scale_up_restarts_gang_with_new_world(cluster, tmp_path):
    """Coordinated scale-up (扩容, k8s-operator.md:1): raising Worker replicas on a running job
    replaces every pod of the old world under a new generation; the new gang's TF_CONFIG lists the
    larger cluster and training resumes from the chief's checkpoint instead of starting over."""
    import time
    c = cluster.client
    ck = str(tmp_path / "ck")
    args = _args(ck, steps=40) + ["--step-sleep", "0.1"]
    c.create(_job("elastic", {"Chief": _rs(1, args), "Worker": _rs(1, args)}))
    dl = time.time() + 120
    while time.time() < dl:
        try:
            if any(e["event"] == "checkpoint" for e in _events(c.logs("elastic-chief-0"))):
                break
        except Exception:
            pass
        time.sleep(0.2)
    else:
        raise AssertionError("chief never checkpointed")
    c.patch("tfjobs", "elastic", {"spec": {"tfReplicaSpecs": {"Worker": {"replicas": 2}}}})
    j = c.wait_tfjob("elastic", timeout=300)
    st = j["status"]
    assert tfjob_condition(j) == "Succeeded", st
    assert st.get("resizeCount") == 1 and not st.get("restartCount"), st
    assert any(cd["type"] == "Restarting" and cd["reason"] == "TFJobResized" for cd in st["conditions"]), st
    pod = c.get("pods", "elastic-worker-1")
    assert pod["metadata"]["annotations"]["tfk.io/world"] == "Chief=1,Worker=2"
    env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0]["env"]}
    assert len(json.loads(env["TF_CONFIG"])["cluster"]["worker"]) == 2
    assert env.get("TFK_RESTART_GENERATION") == "1"
    ev = _events(c.logs("elastic-chief-0"))
    restored = [e for e in ev if e["event"] == "restored"]
    start = [e for e in ev if e["event"] == "start"][-1]
    assert restored and restored[-1]["step"] >= 4, ev[:5]
    assert start["workers"] == 3 and start["start_step"] == restored[-1]["step"]
    assert [e for e in ev if e["event"] == "done"][-1]["step"] == 40


def test_checkpoint_disk_full_fails_clearly_keeps_previous(cluster, tmp_path):
    """Disk failure (k8s-operator.md:5): the step-8 checkpoint write hits ENOSPC (injected in the
    native bundle writer); the job fails with a clear CheckpointWriteFailed message, no partial
    files are left, and the `checkpoint` state still names the intact step-4 checkpoint."""
    import glob
    c = cluster.client
    ck = str(tmp_path / "ck")
    c.create(_job("diskfull", {"Chief": _rs(1, _args(ck, steps=12), [("TFK_FAULT_CKPT_ENOSPC", "model.ckpt-8")])}))
    j = c.wait_tfjob("diskfull", timeout=180)
    assert tfjob_condition(j) == "Failed", j["status"]
    ev = _events(c.logs("diskfull-chief-0"))
    err = [e for e in ev if e["event"] == "error"]
    assert err and err[-1]["kind"] == "checkpoint" and "disk full" in err[-1]["message"], ev[-3:]
    state = open(os.path.join(ck, "checkpoint")).read()
    assert 'model_checkpoint_path: "model.ckpt-4"' in state, state
    assert os.path.exists(os.path.join(ck, "model.ckpt-4.index"))
    assert not glob.glob(os.path.join(ck, "model.ckpt-8*")) and not glob.glob(os.path.join(ck, "*.tmp*"))
    pod = c.get("pods", "diskfull-chief-0")
    term = pod["status"]["containerStatuses"][0]["state"]["terminated"]
    assert term["exitCode"] == 1 and "CheckpointWriteFailed" in term.get("message", ""), term
