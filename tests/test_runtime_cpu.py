"""In-pod runtime on CPU (gloo): TF_CONFIG resolution, the train entrypoint, MWMS vs
ParameterServer equivalence, checkpoint/resume, evaluator, fault-injection exit codes.
Reference behaviour: SURVEY §3.3 (TF_CONFIG contract), D1-D5 (strategies), D10 (checkpoints)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, free_port
from tensorflow_k8s_amd.parallel import cluster

PY = sys.executable


def _env(extra=None):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT
    e["TFK_LOCAL_DNS"] = "1"
    e.pop("TF_CONFIG", None)
    e.update(extra or {})
    return e


def _launch(tasks, cluster_spec, args, tmp, extra_env=None, timeout=240):
    """Run one process per (type, index) with TF_CONFIG; returns {task: (rc, [json events], text)}."""
    procs = {}
    for ty, ix in tasks:
        tf = {"cluster": cluster_spec, "task": {"type": ty, "index": ix}}
        env = _env({"TF_CONFIG": json.dumps(tf), **(extra_env or {})})
        log = open(os.path.join(tmp, f"{ty}-{ix}.log"), "w")
        procs[(ty, ix)] = (subprocess.Popen([PY, "-m", "tensorflow_k8s_amd.runtime.train"] + args, env=env,
                                            stdout=log, stderr=subprocess.STDOUT, cwd=tmp), log)
    out = {}
    for k, (p, log) in procs.items():
        try:
            rc = p.wait(timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            rc = -9
        log.close()
        text = open(log.name).read()
        ev = [json.loads(l) for l in text.splitlines() if l.startswith("{")]
        out[k] = (rc, ev, text)
    return out


def _final_loss(events):
    return [e for e in events if e.get("event") == "done"][-1]["loss"]


# ---------------------------------------------------------------------------- TF_CONFIG
def test_resolve_tf_config_ranks():
    spec = {"cluster": {"chief": ["j-chief-0.ns.svc:2222"], "worker": ["j-worker-0.ns.svc:2222", "j-worker-1.ns.svc:2222"],
                        "ps": ["j-ps-0.ns.svc:2222"]}, "task": {"type": "worker", "index": 1}}
    info = cluster.resolve({"TF_CONFIG": json.dumps(spec), "TFK_LOCAL_DNS": "1"})
    assert (info.rank, info.world_size) == (2, 4)
    assert info.worker_ranks == [0, 1, 2] and info.ps_ranks == [3]
    assert (info.master_addr, info.master_port) == ("127.0.0.1", 2222)
    info = cluster.resolve({"TF_CONFIG": json.dumps({**spec, "task": {"type": "ps", "index": 0}})})
    assert info.is_ps and info.rank == 3 and info.master_addr == "j-chief-0.ns.svc"
    ev = cluster.resolve({"TF_CONFIG": json.dumps({**spec, "task": {"type": "evaluator", "index": 0}})})
    assert ev.is_evaluator and ev.rank == -1
    # v1alpha1 "master" is the chief; no chief -> worker 0 leads
    m = cluster.resolve({"TF_CONFIG": json.dumps({"cluster": {"master": ["m:1"], "worker": ["w:2"]},
                                                  "task": {"type": "master", "index": 0}})})
    assert m.is_chief and m.master_port == 1
    w = cluster.resolve({"TF_CONFIG": json.dumps({"cluster": {"worker": ["w0:5", "w1:6"]},
                                                  "task": {"type": "worker", "index": 0}})})
    assert w.is_chief and w.master_port == 5
    with pytest.raises(ValueError):
        cluster.resolve({"TF_CONFIG": json.dumps({"cluster": {"worker": ["a:1"]}, "task": {"type": "worker", "index": 3}})})
    t = cluster.resolve({"WORLD_SIZE": "4", "RANK": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1234"})
    assert t.source == "torchrun" and t.rank == 2 and t.world_size == 4


# ---------------------------------------------------------------------------- train entrypoint
BASE = ["--model", "lenet", "--steps", "12", "--batch", "16", "--device", "cpu", "--log-every", "4"]


def test_single_process_trains_and_checkpoints(tmp_path, native_ext):
    ck = str(tmp_path / "ck")
    r = subprocess.run([PY, "-m", "tensorflow_k8s_amd.runtime.train"] + BASE + ["--checkpoint-dir", ck,
                       "--checkpoint-every", "4", "--keep", "2"], env=_env(), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    ev = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    losses = [e["loss"] for e in ev if e["event"] == "train"]
    assert losses[-1] < losses[0]
    # keep=2 -> only the two newest bundles remain, state file points at the final one
    idx = sorted(f for f in os.listdir(ck) if f.endswith(".index"))
    assert idx == ["model.ckpt-12.index", "model.ckpt-8.index"]
    from tensorflow_k8s_amd.ops._lib import lib
    latest, allp = lib().ckpt_state_read(ck)
    assert latest == "model.ckpt-12" and allp == ["model.ckpt-8", "model.ckpt-12"]
    t = lib().ckpt_read(os.path.join(ck, "model.ckpt-12"))
    assert tuple(t["conv1/kernel"].shape) == (5, 5, 1, 6)          # TF HWIO, real channels only
    assert tuple(t["fc1/kernel"].shape) == (400, 120)              # dense [in, out]
    assert tuple(t["conv1/kernel/Momentum"].shape) == (5, 5, 1, 6)  # optimizer slot, TF naming
    assert int(t["global_step"]) == 12


def test_mwms_equals_sync_ps_and_resume_is_exact(tmp_path, native_ext):
    """2-worker MWMS (gloo all-reduce) and sync ParameterServer (2 ps shards) apply the same mean
    gradient -> identical losses; a run resumed from the step-8 checkpoint reproduces the
    uninterrupted run exactly (checkpoint carries weights, slots, BN-free LeNet, global_step)."""
    p = free_port()
    mw = _launch([("chief", 0), ("worker", 0)], {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"]},
                 BASE + ["--checkpoint-dir", str(tmp_path / "a"), "--checkpoint-every", "4", "--comm-dtype", "f32"],
                 str(tmp_path))
    assert all(v[0] == 0 for v in mw.values()), {k: v[2][-1500:] for k, v in mw.items()}
    p = free_port()
    ps = _launch([("chief", 0), ("worker", 0), ("ps", 0), ("ps", 1)],
                 {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"], "ps": ["p0.svc:1", "p1.svc:1"]},
                 BASE, str(tmp_path))
    assert all(v[0] == 0 for v in ps.values()), {k: v[2][-1500:] for k, v in ps.items()}
    a, b = _final_loss(mw[("chief", 0)][1]), _final_loss(ps[("chief", 0)][1])
    assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (a, b)
    assert [e for e in ps[("ps", 1)][1] if e["event"] == "done"][0]["updates"] == 12
    # resume: delete the newer checkpoints, rerun -> starts at 8, same final loss
    ck = tmp_path / "a"
    for f in os.listdir(ck):
        if "-12." in f:
            os.remove(ck / f)
    (ck / "checkpoint").write_text('model_checkpoint_path: "model.ckpt-8"\nall_model_checkpoint_paths: "model.ckpt-8"\n')
    os.remove(ck / "DONE")
    p = free_port()
    rs = _launch([("chief", 0), ("worker", 0)], {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"]},
                 BASE + ["--checkpoint-dir", str(ck), "--comm-dtype", "f32"], str(tmp_path))
    ev = rs[("chief", 0)][1]
    assert [e for e in ev if e["event"] == "start"][0]["start_step"] == 8
    assert abs(_final_loss(ev) - a) <= 1e-6 * max(1.0, abs(a))


def test_async_ps_and_evaluator(tmp_path, native_ext):
    p = free_port()
    ck = str(tmp_path / "ck")
    spec = {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"], "ps": ["p.svc:1"], "evaluator": ["e.svc:1"]}
    out = _launch([("chief", 0), ("worker", 0), ("ps", 0), ("evaluator", 0)], spec,
                  BASE + ["--ps-mode", "async", "--checkpoint-dir", ck, "--checkpoint-every", "4",
                          "--eval-timeout", "120"], str(tmp_path))
    assert all(v[0] == 0 for v in out.values()), {k: v[2][-1500:] for k, v in out.items()}
    assert [e for e in out[("ps", 0)][1] if e["event"] == "done"][0]["updates"] == 24  # 12 steps x 2 workers
    evs = [e for e in out[("evaluator", 0)][1] if e["event"] == "eval"]
    assert evs and evs[-1]["step"] == 12 and 0.0 <= evs[-1]["accuracy"] <= 1.0


@pytest.mark.parametrize("code", [1, 137])
def test_fault_injection_exit_codes(tmp_path, code):
    r = subprocess.run([PY, "-m", "tensorflow_k8s_amd.runtime.train"] + BASE,
                       env=_env({"TFK_FAULT_AT_STEP": "3", "TFK_FAULT_EXIT": str(code)}), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == (-9 if code == 137 else code)
    # a later restart generation does not fault again
    r = subprocess.run([PY, "-m", "tensorflow_k8s_amd.runtime.train"] + BASE,
                       env=_env({"TFK_FAULT_AT_STEP": "3", "TFK_FAULT_EXIT": str(code), "TFK_RESTART_GENERATION": "1"}),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0


def test_checkpoint_manager_roundtrip_exact(tmp_path, native_ext):
    from tensorflow_k8s_amd.models.resnet import ResNet
    from tensorflow_k8s_amd.runtime.checkpoint import CheckpointManager
    from tensorflow_k8s_amd.runtime.optimizer import AdamW
    m = ResNet(50, stages=[1, 1, 1, 1], width=16, num_classes=10).to("cpu", seed=3)
    opt = AdamW(m.arena, 1e-3)
    # real (non-padding) elements: alignment gaps and zero-padded channels are not TF variables
    real = torch.zeros(m.arena.numel, dtype=torch.bool)
    for p in m.arena.params:
        ones = torch.ones(p.spec.shape)
        if p.spec.post_init is not None:
            ones = p.spec.post_init(ones)
        real[p.offset:p.offset + p.numel] = ones.reshape(-1) != 0
    for s in opt.slot_names:
        m.arena.slot(s).normal_().mul_(real)
    m.arena.buffers[0].tensor.normal_()
    mgr = CheckpointManager(str(tmp_path), max_to_keep=3)
    mgr.save(m.arena, opt, step=7)
    mgr.wait()
    m2 = ResNet(50, stages=[1, 1, 1, 1], width=16, num_classes=10).to("cpu", seed=99)
    opt2 = AdamW(m2.arena, 1e-3)
    assert mgr.restore(m2.arena, opt2) == 7 and opt2.step_count == 7
    assert torch.equal(m.arena.master, m2.arena.master)
    for s in opt.slot_names:
        assert torch.equal(m.arena.slot(s), m2.arena.slot(s))
    assert torch.equal(m.arena.buffers[0].tensor, m2.arena.buffers[0].tensor)
    # stem kernel stored with the 3 real input channels, HWIO
    from tensorflow_k8s_amd.ops._lib import lib
    t = lib().ckpt_read(str(tmp_path / "model.ckpt-7"), ["conv1/kernel"])
    assert tuple(t["conv1/kernel"].shape) == (7, 7, 3, 16)
    w = m.conv1.w.master.numpy()  # OHWI
    np.testing.assert_array_equal(t["conv1/kernel"].numpy(), np.transpose(w, (1, 2, 3, 0))[:, :, :3, :])


def test_collective_ps_transport_matches_mwms(tmp_path, native_ext):
    """transport=rccl (bucketed reduce -> per-bucket owner update -> broadcast on per-shard
    communicators; run here over gloo collectives) gives the same trajectory as MWMS, including the
    chief's checkpoint fetch of the ps-held slots."""
    p = free_port()
    f32 = ["--comm-dtype", "f32"]
    mw = _launch([("chief", 0), ("worker", 0)], {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"]}, BASE + f32,
                 str(tmp_path))
    assert all(v[0] == 0 for v in mw.values()), {k: v[2][-1500:] for k, v in mw.items()}
    p = free_port()
    ck = str(tmp_path / "ck")
    out = _launch([("chief", 0), ("worker", 0), ("ps", 0), ("ps", 1)],
                  {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"], "ps": ["p0.svc:1", "p1.svc:1"]},
                  BASE + f32 + ["--ps-transport", "rccl", "--checkpoint-dir", ck, "--checkpoint-every", "4",
                                "--bucket-mb", "0.01"], str(tmp_path))  # several buckets per shard
    assert all(v[0] == 0 for v in out.values()), {k: v[2][-1500:] for k, v in out.items()}
    a, b = _final_loss(mw[("chief", 0)][1]), _final_loss(out[("chief", 0)][1])
    assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (a, b)
    from tensorflow_k8s_amd.ops._lib import lib
    t = lib().ckpt_read(os.path.join(ck, "model.ckpt-12"))
    assert float(t["fc1/kernel/Momentum"].abs().sum()) > 0  # slots came from the ps shards


def test_collective_ps_bf16_wire_tracks_f32(tmp_path, native_ext):
    """Collective PS with bf16 on the wire both ways (bf16 gradient reduce, bf16 compute-copy
    broadcast of the weight-decayed buckets, f32 no-decay buckets): 1 PS / 2 workers, the loss
    trajectory stays within 1 % of the f32-wire run, is not bit-identical (the bf16 path ran), and
    the per-step wire volume is reported ~half of f32."""
    traj, wire = {}, {}
    for dt in ("f32", "bf16"):
        p = free_port()
        out = _launch([("chief", 0), ("worker", 0), ("ps", 0)],
                      {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"], "ps": ["p0.svc:1"]},
                      BASE[:-1] + ["1", "--ps-transport", "rccl", "--comm-dtype", dt, "--bucket-mb", "0.02", "--lr", "0.02"],
                      str(tmp_path))
        assert all(v[0] == 0 for v in out.values()), {k: v[2][-1500:] for k, v in out.items()}
        ev = out[("chief", 0)][1]
        traj[dt] = [e["loss"] for e in ev if e.get("event") == "train"]
        wire[dt] = [e for e in ev if e.get("event") == "start"][0]["wire_mb_per_step"]
    a, b = traj["f32"], traj["bf16"]
    assert len(a) == len(b) == 12
    assert max(abs(x - y) / abs(x) for x, y in zip(a, b)) <= 1e-2, traj
    assert a != b, traj
    assert 0.45 < wire["bf16"] / wire["f32"] < 0.6, wire


def test_collective_ps_lr_schedule_matches_mwms(tmp_path, native_ext):
    """LR warmup + cosine decay with the collective PS's bucket-by-bucket owner updates: the global
    step (and so the learning rate / bias corrections) advances once per step however many buckets
    a shard has (Optimizer.step_region), so the trajectory equals MWMS under the same schedule."""
    sched = ["--warmup-steps", "3", "--lr-schedule", "cosine", "--comm-dtype", "f32", "--optimizer", "adamw",
             "--lr", "0.01"]
    p = free_port()
    mw = _launch([("chief", 0), ("worker", 0)], {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"]}, BASE + sched,
                 str(tmp_path))
    assert all(v[0] == 0 for v in mw.values()), {k: v[2][-1500:] for k, v in mw.items()}
    p = free_port()
    out = _launch([("chief", 0), ("worker", 0), ("ps", 0), ("ps", 1)],
                  {"chief": [f"c.svc:{p}"], "worker": ["w.svc:1"], "ps": ["p0.svc:1", "p1.svc:1"]},
                  BASE + sched + ["--ps-transport", "rccl", "--bucket-mb", "0.01"], str(tmp_path))
    assert all(v[0] == 0 for v in out.values()), {k: v[2][-1500:] for k, v in out.items()}
    # the chief's own final loss (the logged train losses are a worker mean under MWMS only). Not
    # bit-exact: the CPU AdamW update of a shard/bucket slice vs the whole arena rounds a few tail
    # elements 1 ulp differently (vectorized vs scalar remainder loops) and Adam's 1/sqrt(v)
    # amplifies that over 12 steps (~0.15 %); a step-count or schedule error would show as a
    # whole-lr-factor difference (warmup lr(0) is 1/3 of lr(2)).
    a, b = _final_loss(mw[("chief", 0)][1]), _final_loss(out[("chief", 0)][1])
    assert abs(a - b) <= 5e-3 * max(1.0, abs(a)), (a, b)


@pytest.mark.parametrize("device_schedule", [False, True])
def test_step_region_advances_once_per_global_step(device_schedule):
    """Three region updates per global step (PS buckets) == one whole-arena update, host or device
    LR schedule (warmup), AdamW bias corrections included."""
    from tensorflow_k8s_amd.models import build_model
    from tensorflow_k8s_amd.runtime.optimizer import AdamW, LRSchedule
    sched = LRSchedule(0.01, warmup=3, total=8, kind="cosine")
    res = []
    for split in (False, True):
        m = build_model("lenet").to("cpu", seed=1)
        opt = AdamW(m.arena, sched)
        if device_schedule:
            opt.enable_device_schedule()
        n = m.arena.numel
        cuts = [0, n // 3 // 64 * 64, 2 * n // 3 // 64 * 64, n]
        for s in range(6):
            g = torch.Generator().manual_seed(s)
            m.arena.grad.copy_(torch.randn(n, generator=g))
            if not split:
                opt.step()
                continue
            for k in range(3):
                opt.region = (cuts[k], cuts[k + 1])
                opt.step_region(advance=k == 0)
            opt.region = None
        res.append((m.arena.master.clone(), opt.sync_step()))
    assert res[0][1] == res[1][1] == 6
    torch.testing.assert_close(res[0][0], res[1][0], rtol=1e-6, atol=1e-7)


def test_gloo_ps_task_survives_short_watchdog(tmp_path, native_ext):
    """a gloo parameter-server task blocks in recv between worker pushes; with the
    watchdog armed (here 2 s) it must beat on every command it receives, so a healthy job that runs
    longer than the timeout (12 paced steps, ~4 s) ends 0 on every task -- not 143 on the ps."""
    p = free_port()
    out = _launch([("chief", 0), ("ps", 0)], {"chief": [f"c.svc:{p}"], "ps": ["p0.svc:1"]},
                  BASE + ["--watchdog-timeout", "2", "--step-sleep", "0.35"], str(tmp_path))
    assert all(v[0] == 0 for v in out.values()), {k: v[2][-1500:] for k, v in out.items()}
    assert not any(e.get("kind") == "watchdog" for v in out.values() for e in v[1])
    assert [e for e in out[("ps", 0)][1] if e["event"] == "done"][0]["updates"] == 12


def test_streams_reset_drops_queued_weight_gradients():
    """a capture that raises mid-backward leaves deferred weight-gradient closures
    queued; StepRunner's fallback path calls streams.reset() so none of them runs in a later step."""
    from tensorflow_k8s_amd.runtime import streams
    ran = []
    streams._pending.append((lambda: ran.append(1), (torch.zeros(1),)))
    streams._keep.append(torch.zeros(1))
    streams.reset()
    streams.flush(force=True)
    assert ran == [] and streams._pending == [] and streams._keep == []
