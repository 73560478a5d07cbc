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
