"""BERT / Transformer executors on the GPU (HIP kernels) vs the CPU reference path of the same
executor (fp32 torch ops), tiny configs, identical dropout masks (hash RNG shared by both)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.float().reshape(-1).cpu(), b.float().reshape(-1).cpu()
    return float(a @ b / (a.norm() * b.norm() + 1e-20))


def _grads(model_fn, batch_fn, dev):
    m = model_fn().to(dev, seed=11)
    batch = batch_fn(m, dev)
    loss, _ = m.forward_backward(*batch)
    return float(loss.mean()), {p.name: p.grad.detach().float().cpu().clone() for p in m.arena.params}


@pytest.mark.parametrize("dropout", [False, True])
@pytest.mark.parametrize("which", ["bert", "transformer"])
def test_gpu_matches_cpu_executor(which, dropout):
    if which == "bert":
        from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining

        def mk():
            c = BertConfig.tiny()
            if not dropout:
                c.hidden_dropout = c.attn_dropout = 0.0
            return BertForPreTraining(c)
    else:
        from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig

        def mk():
            c = TransformerConfig.tiny()
            if not dropout:
                c.dropout = c.attn_dropout = c.relu_dropout = 0.0
            return Transformer(c)
    bfn = lambda m, dev: m.synthetic_batch(4, dev, seed=5)
    lc, gc = _grads(mk, bfn, "cpu")
    lg, gg = _grads(mk, bfn, "cuda")
    assert abs(lc - lg) / abs(lc) < 2e-2, (lc, lg)
    bad = [(n, round(_cos(gg[n], gc[n]), 4)) for n in gc if gc[n].norm() > 1e-6 and _cos(gg[n], gc[n]) < 0.97]
    assert not bad, bad


@pytest.mark.parametrize("which", ["bert-base", "transformer-big"])
def test_full_size_step_runs(which):
    from tensorflow_k8s_amd.models import build_model
    from tensorflow_k8s_amd.runtime.optimizer import LAMB, AdamW
    m = build_model(which).to("cuda")
    opt = (LAMB if which.startswith("bert") else AdamW)(m.arena, 1e-4)
    batch = m.synthetic_batch(8, "cuda", seed=1)
    losses = []
    for _ in range(3):
        loss, _ = m.forward_backward(*batch)
        opt.step()
        losses.append(float(loss.mean()))
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert losses[-1] < losses[0] + 0.5
