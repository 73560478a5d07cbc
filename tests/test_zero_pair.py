"""CPU check: LayerNorm dgamma/dbeta zeroing merges into one fill only for adjacent arena views."""
import torch

from tensorflow_k8s_amd.ops.transformer import _zero_pair


def test_zero_pair_adjacent_and_gapped():
    buf = torch.ones(20)
    _zero_pair(buf[2:8], buf[8:14])
    assert buf[2:14].abs().sum() == 0 and buf[:2].sum() == 2 and buf[14:].sum() == 6
    buf = torch.ones(20)
    _zero_pair(buf[2:8], buf[9:15])  # gap: two fills, the gap element untouched
    assert buf[8] == 1 and buf[2:8].abs().sum() == 0 and buf[9:15].abs().sum() == 0
    a, b = torch.ones(4), torch.ones(4)  # separate storages
    _zero_pair(a, b)
    assert a.abs().sum() == 0 and b.abs().sum() == 0


def test_zero_pair_reversed_order_and_real_layernorm():
    calls = []
    buf = torch.ones(20)
    orig = torch.Tensor.zero_

    def spy(self):
        calls.append(self.numel())
        return orig(self)
    torch.Tensor.zero_ = spy
    try:
        _zero_pair(buf[8:14], buf[2:8])  # b precedes a
    finally:
        torch.Tensor.zero_ = orig
    assert calls == [12] and buf[2:14].abs().sum() == 0 and buf[:2].sum() == 2
    # a real model's LayerNorm gamma/beta gradient views are adjacent (beta first): one fill
    from tensorflow_k8s_amd.models import build_model
    m = build_model("bert-base", layers=1, hidden=64, heads=1, intermediate=128, vocab_size=256, seq_len=16).to("cpu")
    ps = m.arena.by_name()
    gam = [n for n in ps if n.endswith("LayerNorm/gamma")][0]
    bet = gam[: -len("gamma")] + "beta"
    g, b = ps[gam], ps[bet]
    assert abs(g.offset - b.offset) == g.numel
    calls.clear()
    torch.Tensor.zero_ = spy
    try:
        _zero_pair(g.grad.view(-1), b.grad.view(-1))
    finally:
        torch.Tensor.zero_ = orig
    assert calls == [g.numel + b.numel]
