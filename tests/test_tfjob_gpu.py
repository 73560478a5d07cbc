"""SURVEY §7.4's end-to-end slice on the MI355X: the native control plane (tfk-cluster: apiserver +
TFJob operator + gang scheduler + kubelet) runs a ResNet-50 TFJob whose pod trains on the
hand-written gfx950 kernels (reference: TFJob lifecycle k8s-operator.md:1, run-to-completion and
restart semantics :44-52, operator-managed TFJob CRUD :228).

* the gang scheduler binds amd.com/gpu 1 -> GPU 0; the kubelet (which never touches HIP: the GPU
  count comes from --gpus) spawns the runtime with HIP_VISIBLE_DEVICES=0;
* the chief trains ResNet-50 (bf16, batch 32 at 128x128 to keep the test short), writes TF-bundle
  checkpoints and the job reaches Succeeded;
* fault case: the pod SIGKILLs itself at step 9 (exit 137, retryable) -> gang restart generation 1
  -> the new pod restores the newest complete checkpoint (step 8 or 4) -> Succeeded.
"""
import json
import os
import time

import pytest

from tensorflow_k8s_amd.control.client import LocalCluster, tfjob_condition

pytestmark = pytest.mark.gpu

TRAIN = ["python3", "-m", "tensorflow_k8s_amd.runtime.train"]


def _job(name, ck, fault=()):
    args = ["--model", "resnet50", "--batch", "32", "--image-size", "128", "--steps", "12", "--device", "cuda",
            "--log-every", "2", "--checkpoint-dir", ck, "--checkpoint-every", "4"]
    c = {"name": "tensorflow", "image": "tfk/runtime", "command": TRAIN, "args": args,
         "env": [{"name": k, "value": v} for k, v in fault],
         "resources": {"limits": {"amd.com/gpu": 1}}}
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"runPolicy": {"backoffLimit": 2, "cleanPodPolicy": "None"},
                     "tfReplicaSpecs": {"Chief": {"replicas": 1, "restartPolicy": "ExitCode",
                                                  "template": {"spec": {"containers": [c]}}}}}}


def _events(text):
    return [json.loads(l) for l in text.splitlines() if l.startswith("{")]


@pytest.fixture
def gpu_cluster(tmp_path, native_ext):
    # prebuilt in-tree (the GPU box does not rebuild the control plane: its objects stay behind)
    from tensorflow_k8s_amd.control.client import BIN
    assert os.access(os.path.join(BIN, "tfk-cluster"), os.X_OK), "build the control plane first (make -C cpp)"
    with LocalCluster(gpus=1, root_dir=str(tmp_path / "cluster")) as c:
        yield c


@pytest.mark.timeout(300)
def test_resnet50_tfjob_trains_on_gpu_and_restarts(gpu_cluster, tmp_path):
    c = gpu_cluster.client
    ck = str(tmp_path / "ck")
    c.create(_job("r50", ck))
    j = c.wait_tfjob("r50", timeout=240)
    assert tfjob_condition(j) == "Succeeded", (j["status"], c.logs("r50-chief-0")[-3000:])
    pod = c.get("pods", "r50-chief-0")
    env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0]["env"]}
    assert json.loads(env["TF_CONFIG"])["task"] == {"type": "chief", "index": 0}
    ev = _events(c.logs("r50-chief-0"))
    start = [e for e in ev if e["event"] == "start"][0]
    assert start["device"].startswith("cuda") and start["model"] == "resnet50", start
    train = [e for e in ev if e["event"] == "train"]
    assert train and all(e["loss"] == e["loss"] for e in train)  # finite
    assert [e for e in ev if e["event"] == "done"][-1]["step"] == 12
    assert os.path.exists(os.path.join(ck, "model.ckpt-12.index"))
    assert "model.ckpt-12" in open(os.path.join(ck, "checkpoint")).read()

    # retryable failure at step 9 -> gang restart -> resume from the newest complete checkpoint
    # (step 8 if its asynchronous write finished before the SIGKILL, else step 4)
    ck2 = str(tmp_path / "ck2")
    c.create(_job("r50f", ck2, fault=[("TFK_FAULT_AT_STEP", "9"), ("TFK_FAULT_EXIT", "137")]))
    j = c.wait_tfjob("r50f", timeout=240)
    st = j["status"]
    assert tfjob_condition(j) == "Succeeded", (st, c.logs("r50f-chief-0")[-3000:])
    assert st.get("restartCount") == 1 and any(cd["type"] == "Restarting" for cd in st["conditions"]), st
    ev = _events(c.logs("r50f-chief-0"))
    restored = [e for e in ev if e["event"] == "restored"]
    assert restored and restored[-1]["step"] in (4, 8), [e for e in ev if e["event"] != "train"]
    assert [e for e in ev if e["event"] == "done"][-1]["step"] == 12


@pytest.mark.timeout(420)
def test_config4_resnet152_chief_evaluator_fault_restart(gpu_cluster, tmp_path):
    """BASELINE config 4 on the MI355X: ResNet-152 Chief (GPU) + Evaluator (same GPU, outside the
    training world). The chief SIGKILLs itself at step 9 (exit 137, retryable) -> gang restart ->
    resume from the newest complete checkpoint -> Succeeded; the evaluator follows the checkpoint
    directory and reports an eval for the final checkpoint, which was written after the restart.
    Both replicas mount the checkpoint volume (persistentVolumeClaim) at /tfk-ckpt."""
    c = gpu_cluster.client
    # the checkpoints live on a declared volume (a PVC-like directory of the kubelet) mounted into
    # the chief and the evaluator at /tfk-ckpt (SURVEY §5.4 storage)
    ck = "/tfk-ckpt/r152"
    vol = [{"name": "ckpt", "persistentVolumeClaim": {"claimName": "r152-ckpt"}}]
    mnt = [{"name": "ckpt", "mountPath": "/tfk-ckpt"}]
    common = ["--model", "resnet152", "--image-size", "64", "--num-classes", "100", "--device", "cuda",
              "--checkpoint-dir", ck]
    chief = {"name": "tensorflow", "image": "tfk/runtime", "command": TRAIN,
             "args": common + ["--batch", "16", "--steps", "12", "--checkpoint-every", "4", "--log-every", "2"],
             "env": [{"name": "TFK_FAULT_AT_STEP", "value": "9"}, {"name": "TFK_FAULT_EXIT", "value": "137"}],
             "resources": {"limits": {"amd.com/gpu": 1}}, "volumeMounts": mnt}
    evaluator = {"name": "tensorflow", "image": "tfk/runtime", "command": TRAIN,
                 "args": common + ["--batch", "8", "--eval-batches", "2", "--eval-timeout", "300"], "volumeMounts": mnt}
    job = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": "r152", "namespace": "default"},
           "spec": {"runPolicy": {"backoffLimit": 2, "cleanPodPolicy": "None"},
                    "tfReplicaSpecs": {
                        "Chief": {"replicas": 1, "restartPolicy": "ExitCode",
                                  "template": {"spec": {"containers": [chief], "volumes": vol}}},
                        "Evaluator": {"replicas": 1, "restartPolicy": "OnFailure",
                                      "template": {"spec": {"containers": [evaluator], "volumes": vol}}}}}}
    c.create(job)
    j = c.wait_tfjob("r152", timeout=360)
    st = j["status"]
    assert tfjob_condition(j) == "Succeeded", (st, c.logs("r152-chief-0")[-3000:])
    assert st.get("restartCount") == 1, st
    ev = _events(c.logs("r152-chief-0"))
    restored = [e for e in ev if e["event"] == "restored"]
    assert restored and restored[-1]["step"] in (4, 8), [e for e in ev if e["event"] != "train"]
    assert [e for e in ev if e["event"] == "done"][-1]["step"] == 12
    start = [e for e in ev if e["event"] == "start"][-1]
    assert start["model"] == "resnet152" and start["restart_generation"] == 1, start
    # the evaluator is not in the training world: TF_CONFIG task only, no cluster slot
    pod = c.get("pods", "r152-evaluator-0")
    env = {e["name"]: e.get("value") for e in pod["spec"]["containers"][0]["env"]}
    tf = json.loads(env["TF_CONFIG"])
    assert tf["task"] == {"type": "evaluator", "index": 0} and "evaluator" not in tf["cluster"], tf
    deadline = time.time() + 120
    evals = []
    while time.time() < deadline:
        evals = [e for e in _events(c.logs("r152-evaluator-0")) if e.get("event") == "eval"]
        if any(e["step"] == 12 for e in evals):
            break
        time.sleep(1)
    assert any(e["step"] == 12 for e in evals), (evals, c.logs("r152-evaluator-0")[-2000:])
    last = [e for e in evals if e["step"] == 12][-1]
    assert last["loss"] == last["loss"] and 0.0 <= last["accuracy"] <= 1.0 and last["examples"] == 16
    host = os.path.join(str(tmp_path), "cluster", "kubelet", "pvc", "default", "r152-ckpt", "r152")
    assert "model.ckpt-12" in open(os.path.join(host, "checkpoint")).read()
