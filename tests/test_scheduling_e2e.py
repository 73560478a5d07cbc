"""Gang scheduler policy end to end through tfk-cluster (CPU; GPUs are accounted, not used):

* priority: with the node full, a TFJob whose schedulingPolicy.priorityClass names a
  scheduling.k8s.io/v1 PriorityClass of higher value is placed before an OLDER default-priority
  job once the GPUs free up;
* topology: the node publishes its GPU->NUMA map (tfk.io/gpu-numa), a 2-pod gang lands on GPUs of
  one NUMA node, and the kubelet pins each container's CPUs to that node's CPU list
  (TFK_CPU_AFFINITY + sched_getaffinity seen from inside the pod).
Reference: gang scheduling of chief/PS/worker pods onto one 8x MI355X node (BASELINE north star),
SURVEY §2 C28.
"""
import json
import os
import time

import pytest

from tensorflow_k8s_amd.control.client import ApiError, LocalCluster, tfjob_condition

PRINT_AFF = ["python3", "-c", "import os, json; print(json.dumps({'aff': sorted(os.sched_getaffinity(0)), "
             "'env': os.environ.get('TFK_CPU_AFFINITY'), 'gpus': os.environ.get('HIP_VISIBLE_DEVICES')}))"]


def _rs(n, cmd, gpus=1):
    return {"replicas": n, "restartPolicy": "Never", "template": {"spec": {"containers": [{
        "name": "tensorflow", "image": "tfk/runtime", "command": cmd, "resources": {"limits": {"amd.com/gpu": gpus}}}]}}}


def _job(name, specs, priority_class=None):
    rp = {"cleanPodPolicy": "None"}
    if priority_class:
        rp["schedulingPolicy"] = {"priorityClass": priority_class}
    return {"apiVersion": "kubeflow.org/v1", "kind": "TFJob", "metadata": {"name": name, "namespace": "default"},
            "spec": {"tfReplicaSpecs": specs, "runPolicy": rp}}


def _bound(c, pod):
    try:
        return bool(c.get("pods", pod).get("spec", {}).get("nodeName"))
    except ApiError:
        return False


def _wait_bound(c, pod, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline and not _bound(c, pod):
        time.sleep(0.1)
    assert _bound(c, pod), pod


def _start_time(c, pod):
    p = c.get("pods", pod)
    for cs in p.get("status", {}).get("containerStatuses", []):
        for st in (cs.get("state", {}), cs.get("lastState", {})):
            for k in ("running", "terminated"):
                if st.get(k, {}).get("startedAt"):
                    return st[k]["startedAt"]
    return None


def test_priority_class_orders_pending_gangs(tmp_path, control_plane_bin):
    with LocalCluster(gpus=2, root_dir=str(tmp_path / "c")) as cl:
        c = cl.client
        c.create({"apiVersion": "scheduling.k8s.io/v1", "kind": "PriorityClass", "metadata": {"name": "urgent"},
                  "value": 100000})
        # the blocker holds both GPUs for ~3 s
        c.create(_job("blocker", {"Chief": _rs(1, ["python3", "-c", "import time; time.sleep(3)"], gpus=2)}))
        _wait_bound(c, "blocker-chief-0")
        ok = ["python3", "-c", "pass"]
        c.create(_job("low", {"Chief": _rs(1, ok, gpus=2)}))             # older, default priority
        time.sleep(1.0)
        c.create(_job("high", {"Chief": _rs(1, ok, gpus=2)}, priority_class="urgent"))
        for name in ("blocker", "low", "high"):
            assert tfjob_condition(c.wait_tfjob(name, timeout=90)) == "Succeeded", name
        assert c.get("pods", "high-chief-0")["spec"].get("priorityClassName") == "urgent"
        th, tl = _start_time(c, "high-chief-0"), _start_time(c, "low-chief-0")
        assert th and tl and th <= tl, (th, tl)


def test_numa_packed_gang_and_cpu_pinning(tmp_path, control_plane_bin):
    ncpu = os.cpu_count() or 2
    if ncpu < 2:
        pytest.skip("needs >= 2 CPUs")
    half = ncpu // 2
    numa_cpus = f"0-{half - 1};{half}-{ncpu - 1}"
    with LocalCluster(gpus=4, root_dir=str(tmp_path / "c"),
                      extra_args=["--gpu-numa", "0,0,1,1", "--numa-cpus", numa_cpus]) as cl:
        c = cl.client
        # the kubelet registers its Node asynchronously after the cluster is up
        deadline = time.time() + 20
        nodes = c.list("nodes", ns=None)
        while not nodes and time.time() < deadline:
            time.sleep(0.2)
            nodes = c.list("nodes", ns=None)
        assert nodes, "kubelet never registered its node"
        node = nodes[0]
        assert node["metadata"]["annotations"]["tfk.io/gpu-numa"] == "0,0,1,1"
        # occupy GPU 0 so domain 0 has one free GPU: the 2-pod gang must pack onto domain 1
        c.create(_job("hold", {"Chief": _rs(1, ["python3", "-c", "import time; time.sleep(4)"])}))
        _wait_bound(c, "hold-chief-0")
        c.create(_job("gang", {"Chief": _rs(1, PRINT_AFF), "Worker": _rs(1, PRINT_AFF)}))
        assert tfjob_condition(c.wait_tfjob("gang", timeout=90)) == "Succeeded"
        dom1 = set(range(half, ncpu))
        for pod in ("gang-chief-0", "gang-worker-0"):
            ids = c.get("pods", pod)["metadata"]["annotations"]["tfk.io/gpu-ids"]
            assert ids in ("2", "3"), (pod, ids)
            out = [json.loads(l) for l in c.logs(pod).splitlines() if l.startswith("{")][-1]
            assert set(out["aff"]) == dom1, out
            assert out["env"] == ",".join(str(x) for x in sorted(dom1))


PRINT_VIS = ["python3", "-c", "import os, json; print(json.dumps({'gpus': os.environ.get('HIP_VISIBLE_DEVICES'), "
             "'local': os.environ.get('TFK_LOCAL_DEVICE')}))"]


def test_gang_visible_gpus_opt_in(tmp_path, control_plane_bin):
    """With the TFJob annotation scheduling.tfk.io/gang-visible-gpus, every gang member sees ALL of
    the gang's GPUs on the node (so RCCL between the pods can use xGMI P2P/IPC) and TFK_LOCAL_DEVICE
    names its own one; without it a pod sees only its own GPU (local device 0)."""
    with LocalCluster(gpus=4, root_dir=str(tmp_path / "c")) as cl:
        c = cl.client
        job = _job("vis", {"Chief": _rs(1, PRINT_VIS), "Worker": _rs(2, PRINT_VIS)})
        job["metadata"]["annotations"] = {"scheduling.tfk.io/gang-visible-gpus": "true"}
        c.create(job)
        c.create(_job("iso", {"Chief": _rs(1, PRINT_VIS)}))
        for n in ("vis", "iso"):
            assert tfjob_condition(c.wait_tfjob(n, timeout=90)) == "Succeeded", n
        own, seen = [], set()
        for pod in ("vis-chief-0", "vis-worker-0", "vis-worker-1"):
            an = c.get("pods", pod)["metadata"]["annotations"]
            out = [json.loads(l) for l in c.logs(pod).splitlines() if l.startswith("{")][-1]
            vis = out["gpus"].split(",")
            assert out["gpus"] == an["tfk.io/gang-gpu-ids"] and len(vis) == 3, (pod, out, an)
            assert vis[int(out["local"])] == an["tfk.io/gpu-ids"], (pod, out, an)
            own.append(an["tfk.io/gpu-ids"])
            seen.add(out["gpus"])
        assert len(set(own)) == 3 and len(seen) == 1  # disjoint own GPUs, one shared visible list
        an = c.get("pods", "iso-chief-0")["metadata"]["annotations"]
        out = [json.loads(l) for l in c.logs("iso-chief-0").splitlines() if l.startswith("{")][-1]
        assert "tfk.io/gang-gpu-ids" not in an and out == {"gpus": an["tfk.io/gpu-ids"], "local": "0"}
