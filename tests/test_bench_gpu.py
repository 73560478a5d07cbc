"""bench.py harness on one MI355X beyond the headline run: the ParameterServerStrategy path
(BASELINE config 3's harness -- ``--strategy ps``) launched by torchrun, here with one GPU worker and
one CPU parameter server (gloo transport, the only PS layout one GPU can host; the 8-GPU
PS=2/worker=6 rccl layout is the same code with ``--ps-transport rccl``), and the forced-comm
MWMS run reporting its RCCL configuration. Reference: SURVEY §2 D5, D12; k8s-operator.md:6."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, free_port

pytestmark = pytest.mark.gpu


def _bench_line(out: str) -> dict:
    return json.loads([l for l in out.splitlines() if l.startswith("{") and '"metric"' in l][-1])


def test_bench_ps_strategy_one_gpu_worker_cpu_ps(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="8")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--model", "resnet50", "--batch", "32", "--steps", "3", "--warmup", "2",
                        "--strategy", "ps", "--ps", "1", "--ps-transport", "gloo"],
                       env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _bench_line(r.stdout)
    assert d["config"]["parallelism"] == "ps1+worker1" and d["config"]["global_batch"] == 32
    assert d["config"]["comm"]["ps_ranks"] == [1] and d["config"]["comm"]["transport"] == "gloo"
    assert d["value"] > 0 and d["steps"] == 3 and d["loss"] is not None


def test_bench_force_comm_reports_rccl(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "resnet50", "--batch", "64",
                        "--steps", "3", "--warmup", "3", "--force-comm"],
                       env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = _bench_line(r.stdout)
    c = d["config"]
    assert c["hipgraph"] is True and c["comm"]["wire_mb_per_step"] > 0
    assert c["comm"]["backend"].startswith("tfk_comm RCCL")
    g = c["comm"]["guards"]
    assert g["comm_self_test"]["ok"] is True and g["capture_probe"] == "ok" and "capture_fallback" not in g
    assert g["watchdog_s"] == 300.0


def _run_bench(tmp_path, extra, env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "resnet50", "--batch", "32",
                        "--steps", "2", "--warmup", "3", "--force-comm"] + extra,
                       env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return _bench_line(r.stdout)


def test_bench_injected_capture_failures_fall_back_to_eager(tmp_path):
    """First-N-GPU-run guards on the GPU (runtime/guard.py): an injected capture-probe failure and
    an injected failure of the real step's capture both make the run fall back to eager steps
    in-process; the JSON says why, and the loss equals a plain eager run's (same data, same init)."""
    eager = _run_bench(tmp_path, ["--graph", "0"])
    assert eager["config"]["hipgraph"] is False and eager["config"]["comm"]["guards"]["capture_probe"] == "off"
    probe = _run_bench(tmp_path, [], {"TFK_FAULT_CAPTURE": "1"})
    gp = probe["config"]["comm"]["guards"]
    assert probe["config"]["hipgraph"] is False and "injected probe capture failure" in gp["capture_probe"]
    step = _run_bench(tmp_path, [], {"TFK_FAULT_CAPTURE": "step"})
    gs = step["config"]["comm"]["guards"]
    assert gs["capture_probe"] == "ok" and "injected step capture failure" in gs["capture_fallback"]
    assert step["config"]["hipgraph"] is False
    for d in (probe, step):
        assert abs(d["loss"] - eager["loss"]) <= 1e-3 * abs(eager["loss"]), (d["loss"], eager["loss"])


def test_bench_collective_ps_colocated_one_gpu(tmp_path):
    """The collective (RCCL) parameter-server transport on one GPU: worker 0 owns the only shard
    (colocated owner), so the bucketed reduce -> unpack -> step_region -> broadcast path runs on GPU
    tensors inside the captured worker step."""
    d = _run_bench(tmp_path, ["--strategy", "ps", "--ps-transport", "rccl"])
    c = d["config"]
    assert c["parallelism"] == "ps1+worker1" and c["comm"]["transport"] == "rccl"
    assert c["comm"]["wire_mb_per_step"] > 0 and c["comm"]["buckets"] > 0
    assert c["hipgraph"] is True and d["loss"] is not None and d["loss"] == d["loss"]


def _run_model(tmp_path, model, extra, batch=None, force=True):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--model", model, "--steps", "6", "--warmup", "3",
           "--report-update"] + (["--force-comm"] if force else []) + (["--batch", str(batch)] if batch else []) + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return _bench_line(r.stdout)


def _captured_ok(d):
    c = d["config"]
    g = c["comm"]["guards"]
    assert c["hipgraph"] is True and "capture_fallback" not in g, g
    assert g["emb_guard"] == 0, g  # the bucketed embedding backward saw consistent counts every step


def test_bench_collective_ps_bert_captured_matches_eager(tmp_path):
    """BASELINE config 3's model on the collective (RCCL) parameter-server transport, colocated owner,
    the whole worker step (reduce -> unpack -> step_region -> broadcast included) replayed from one
    hipGraph -- the step that faulted on replay in round 4 (a hipMemsetAsync captured in the
    embedding backward: perf_log_r5.md). Six steps captured vs eager: same loss, same master update."""
    ps = ["--strategy", "ps", "--ps-transport", "rccl"]
    graph = _run_model(tmp_path, "bert-base", ps)
    eager = _run_model(tmp_path, "bert-base", ps + ["--graph", "0"])
    _captured_ok(graph)
    assert eager["config"]["hipgraph"] is False
    assert abs(graph["loss"] - eager["loss"]) <= 1e-4 * abs(eager["loss"]), (graph["loss"], eager["loss"])
    assert abs(graph["update_norm"] - eager["update_norm"]) <= 1e-3 * eager["update_norm"]
    assert graph["update_norm"] > 0


def test_bench_transformer_big_captured_with_collectives(tmp_path):
    """Transformer-big with the RCCL collectives forced on at world size 1 (MWMS all-reduce buckets,
    then the collective PS path): both steps replay from one hipGraph without the round-4 fault."""
    mw = _run_model(tmp_path, "transformer-big", [])
    _captured_ok(mw)
    ps = _run_model(tmp_path, "transformer-big", ["--strategy", "ps", "--ps-transport", "rccl"])
    _captured_ok(ps)
    assert ps["config"]["comm"]["transport"] == "rccl" and ps["config"]["comm"]["buckets"] > 1
    # the same model, data and optimizer: the PS update equals the MWMS one at world size 1
    assert abs(ps["loss"] - mw["loss"]) <= 1e-3 * abs(mw["loss"]), (ps["loss"], mw["loss"])


@pytest.mark.parametrize("wire", ["f32", "bf16"])
def test_forced_comm_captured_update_equals_no_comm(tmp_path, wire):
    """World-size-1 MWMS with the RCCL bucket all-reduces forced on, captured: the bucket launches
    make the comm stream (not the compute stream) wait on the side-stream weight gradients
    (runtime/streams.py producers) and pack the bf16 wire there. The master update must equal the
    no-comm captured step's to the step's own run-to-run spread on the f32 wire (a 1-rank sum is the
    identity; the BN statistics' f32 atomics make two identical runs differ by ~1e-4), to bf16
    rounding of the gradients on the bf16 wire. A bucket launched before one of its weight gradients
    finished would reduce a stale slice and change the update by far more."""
    nc = _run_model(tmp_path, "resnet50", ["--comm-dtype", wire], batch=64, force=False)
    fc = _run_model(tmp_path, "resnet50", ["--comm-dtype", wire], batch=64)
    assert nc["config"]["hipgraph"] and fc["config"]["hipgraph"]
    assert fc["config"]["comm"]["wire_mb_per_step"] > 0 and nc["config"]["comm"]["wire_mb_per_step"] == 0
    tol = 3e-4 if wire == "f32" else 2e-2  # run-to-run spread of the step itself: ~1e-4 (f32 atomics)
    assert abs(fc["update_norm"] - nc["update_norm"]) <= tol * nc["update_norm"], (fc["update_norm"], nc["update_norm"])
    assert abs(fc["loss"] - nc["loss"]) <= tol * abs(nc["loss"]) + 1e-6, (fc["loss"], nc["loss"])
