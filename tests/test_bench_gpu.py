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
