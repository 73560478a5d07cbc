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
