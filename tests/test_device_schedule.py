"""hipGraph-safe optimizer schedules (runtime/trainer.py): the learning rate, step
counter and Adam bias corrections live on the device (Optimizer.enable_device_schedule), so a
captured step replays the right update every time. CPU: the device-schedule path equals the host
path step for step; GPU: a graph-captured LeNet step with AdamW + warmup/cosine equals eager."""
import pytest
import torch

from tensorflow_k8s_amd.models import build_model, synthetic_batch
from tensorflow_k8s_amd.runtime.optimizer import LAMB, SGD, AdamW, LRSchedule
from tensorflow_k8s_amd.runtime.trainer import GraphUnsafe, StepRunner, graph_hazards


def _fake_grads(arena, step):
    g = torch.Generator().manual_seed(100 + step)
    arena.grad.copy_(torch.randn(arena.grad.shape, generator=g).to(arena.grad.device))


@pytest.mark.parametrize("cls", [SGD, AdamW, LAMB])
def test_device_schedule_matches_host_cpu(cls):
    sched = LRSchedule(0.01, warmup=3, total=12, kind="cosine", end_lr=0.001)
    runs = []
    for dev_sched in (False, True):
        m = build_model("lenet").to("cpu")
        opt = cls(m.arena, sched)
        if dev_sched:
            opt.enable_device_schedule()
        for s in range(12):
            _fake_grads(m.arena, s)
            opt.step()
        runs.append((m.arena.master.clone(), opt.sync_step()))
    assert runs[1][1] == runs[0][1] == 12
    assert torch.allclose(runs[0][0], runs[1][0], rtol=1e-5, atol=1e-7)


def test_device_schedule_state_dict_roundtrip():
    m = build_model("lenet").to("cpu")
    opt = AdamW(m.arena, LRSchedule(1e-3, warmup=2))
    opt.enable_device_schedule()
    for s in range(5):
        _fake_grads(m.arena, s)
        opt.step()
    assert opt.state_dict() == {"step": 5}
    opt.load_state_dict({"step": 9})
    assert int(opt._dev["step"][0]) == 9


def test_graph_refuses_host_dropout_seeds():
    model = build_model("bert-base", layers=1, hidden=64, heads=1, intermediate=128, vocab_size=256, seq_len=16)
    assert graph_hazards(model)
    assert not graph_hazards(build_model("lenet"))


@pytest.mark.gpu
def test_graph_capture_replays_schedule_gpu():
    dev = torch.device("cuda", 0)
    sched = LRSchedule(2e-3, warmup=4, total=20, kind="cosine", end_lr=1e-4)
    finals = []
    for graph in (False, True):
        torch.manual_seed(0)
        m = build_model("lenet").to(dev)
        opt = AdamW(m.arena, sched)
        batch = synthetic_batch(m, 64, dev, seed=3)
        r = StepRunner(m, opt, None, batch, use_graph=graph)
        for _ in range(12):
            r.step()
        torch.cuda.synchronize()
        finals.append((m.arena.master.clone(), opt.sync_step(), r.last_loss()))
    assert finals[1][1] == 12  # the device counter advanced on every replay
    assert torch.allclose(finals[0][0], finals[1][0], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_graph_unsafe_model_raises_gpu():
    dev = torch.device("cuda", 0)
    model = build_model("bert-base", layers=1, hidden=64, heads=1, intermediate=128, vocab_size=256, seq_len=16).to(dev)
    opt = AdamW(model.arena, 1e-3)
    batch = synthetic_batch(model, 2, dev)
    with pytest.raises(GraphUnsafe):
        StepRunner(model, opt, None, batch, use_graph=True)
