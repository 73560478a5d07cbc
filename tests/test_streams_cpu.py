"""runtime/streams.py on CPU tensors: run_wgrad runs inline (no side stream, nothing kept), and
sync/join are no-ops without CUDA -- the CPU executor and the eager multi-process tests rely on it."""
import torch

from tensorflow_k8s_amd.runtime import streams


def test_run_wgrad_inline_on_cpu(monkeypatch):
    monkeypatch.setattr(streams, "MODE", "1")  # even when forced on, CPU tensors never fork
    out = []
    x = torch.ones(4)
    streams.run_wgrad(lambda: out.append(float(x.sum())), x)
    assert out == [4.0]
    assert streams._keep == []
    streams.sync()
    streams.join()
    assert streams._keep == []


def test_mode_off_runs_inline(monkeypatch):
    monkeypatch.setattr(streams, "MODE", "0")
    out = []
    streams.run_wgrad(lambda: out.append(1), torch.zeros(1))
    assert out == [1]


def test_bucket_launch_never_joins_side_streams_into_main(monkeypatch):
    """MWMS bucket launch: the all-reduce gets the side streams as comm-stream dependencies and the
    bf16 wire pack as a comm-stream producer; the compute stream is never made to wait on the side
    streams (streams.sync is not called) before the optimizer's join."""
    from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
    from tensorflow_k8s_amd.runtime.arena import ParamArena, ParamSpec

    class FakeComm:
        world, rank = 2, 0

        def __init__(self):
            self.calls = []

        def all_reduce(self, t, async_op=False, deps=(), pre=None, **kw):
            self.calls.append((t.numel(), list(deps), pre))
            if pre is not None:
                pre()
            return None
    sentinel = object()
    monkeypatch.setattr(streams, "producers", lambda: [sentinel])
    monkeypatch.setattr(streams, "sync", lambda: (_ for _ in ()).throw(AssertionError("main joined side streams")))
    a = ParamArena()
    for i in range(3):
        a.add(ParamSpec(f"w{i}", (64, 64)))
    a.finalize("cpu", seed=0)
    comm = FakeComm()
    s = MultiWorkerMirroredStrategy(a, comm=comm, bucket_mb=0.01, comm_dtype="bf16")
    s.begin_step()
    a.grad.fill_(1.5)
    for p in sorted(a.params, key=lambda p: -p.offset):
        s._on_ready(p)
    s.finish_step()
    assert comm.calls and all(c[1] == [sentinel] and c[2] is not None for c in comm.calls)
    assert float(s.wire.float().sum()) == 1.5 * s.wire.numel()
