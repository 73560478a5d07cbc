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


def test_device_rng_makes_dropout_models_capturable():
    """Dropout models keep their RNG state on the device -> no graph hazard; a model whose dropout
    seeds would come from the host (no rng_state) is still refused."""
    model = build_model("bert-base", layers=1, hidden=64, heads=1, intermediate=128, vocab_size=256, seq_len=16)
    assert not graph_hazards(model)
    assert not graph_hazards(build_model("transformer-big", enc_layers=1, dec_layers=1, hidden=64, heads=1,
                                         filter_size=128, vocab_size=256, src_len=16, tgt_len=16))
    model.rng_state = None
    assert graph_hazards(model)
    assert not graph_hazards(build_model("lenet"))


def test_device_rng_cpu_reference():
    """rng_advance steps [counter, key] (splitmix64 of counter ^ stream); eff_seed = salt + key while
    the state is registered; the dropout mask follows eff_seed and differs per step and per stream."""
    from tensorflow_k8s_amd.ops import elementwise as E
    st = torch.zeros(2, dtype=torch.int64)
    E.rng_advance(st, 0)
    k1 = int(st[1])
    E.rng_advance(st, 0)
    assert int(st[0]) == 2 and int(st[1]) != k1
    st2 = torch.tensor([1, 0], dtype=torch.int64)
    E.rng_advance(st2, 0)
    assert int(st2[1]) == int(st[1])  # a pure function of (counter, stream)
    st3 = torch.tensor([1, 0], dtype=torch.int64)
    E.rng_advance(st3, 1)
    assert int(st3[1]) != int(st[1])
    x = torch.ones(4096, dtype=torch.bfloat16)
    assert E.eff_seed(5) == 5
    with E.rng_key(st):
        assert E.eff_seed(5) == E._s64(5 + int(st[1]))
        y = E.dropout(x, 0.5, 5)
    keep = E.dropout_keep(E._s64(5 + int(st[1])), 4096, 0.5)
    assert torch.equal(y.float() != 0, keep)
    with E.rng_key(st3):
        y3 = E.dropout(x, 0.5, 5)
    assert not torch.equal(y3, y)


@pytest.mark.gpu
def test_device_rng_kernel_masks_captured_equal_eager_gpu():
    """The dropout kernel with the device key: 5 replays of a captured (rng_advance + dropout) step
    give bit-identical masks to 5 eager steps, every mask differs from the previous one, the key
    matches the CPU reference, and each mask equals the CPU hash reference of salt + key."""
    from tensorflow_k8s_amd.ops import elementwise as E
    dev = torch.device("cuda", 0)
    x = torch.ones(1 << 16, dtype=torch.bfloat16, device=dev)
    out = torch.empty_like(x)

    def step(st):
        E.rng_advance(st, 3)
        with E.rng_key(st):
            out.copy_(E.dropout(x, 0.3, 1234))

    st = torch.zeros(2, dtype=torch.int64, device=dev)
    eager = []
    for _ in range(5):
        step(st)
        eager.append(out.clone())
    st_g = torch.zeros(2, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up (allocations) on a side stream, then reset the state
        step(st_g)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    st_g.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(st_g)
    graphed = []
    for _ in range(5):
        g.replay()
        graphed.append(out.clone())
    torch.cuda.synchronize()
    assert torch.equal(st.cpu(), st_g.cpu()) and int(st_g[0]) == 5
    ref = torch.zeros(2, dtype=torch.int64)
    for i in range(5):
        assert torch.equal(eager[i], graphed[i]), i
        if i:
            assert not torch.equal(graphed[i], graphed[i - 1])
        E.rng_advance(ref, 3)
        keep = E.dropout_keep(E._s64(1234 + int(ref[1])), x.numel(), 0.3)
        assert torch.equal(graphed[i].cpu().float() != 0, keep), i
    assert torch.equal(ref, st.cpu())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bert-base", "transformer-big"])
def test_dropout_model_graph_replay_matches_eager_gpu(name):
    """A dropout-on model step captured in a hipGraph replays the same training as eager steps: the
    device RNG state advances on every replay (same counter and key as eager) and the loss
    trajectory matches (step 1 bit-identical; later steps up to float-atomic reduction order)."""
    dev = torch.device("cuda", 0)
    kw = (dict(layers=2, hidden=128, heads=2, intermediate=256, vocab_size=512, seq_len=64) if name == "bert-base"
          else dict(enc_layers=2, dec_layers=2, hidden=128, heads=2, filter_size=256, vocab_size=512, src_len=32,
                    tgt_len=32))
    runs = []
    for graph in (False, True):
        m = build_model(name, **kw).to(dev, seed=11)
        opt = AdamW(m.arena, 1e-3)
        batch = synthetic_batch(m, 4, dev, seed=5)
        r = StepRunner(m, opt, None, batch, use_graph=graph)
        losses = []
        for _ in range(5):
            r.step()
            losses.append(r.last_loss())
        torch.cuda.synchronize()
        runs.append((losses, m.rng_state.cpu().clone(), r.graph is not None))
    (le, se, _), (lg, sg, captured) = runs
    assert captured and int(se[0]) == 5 and torch.equal(se, sg)
    assert le[0] == lg[0], (le, lg)
    for a, b in zip(le, lg):
        assert abs(a - b) <= 2e-3 * abs(a), (le, lg)
    assert len(set(round(v, 6) for v in lg)) == 5  # fresh masks + updates every replay
