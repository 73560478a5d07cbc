"""Tight GPU-vs-CPU parity of the model executors (VERDICT r1 "tighten GPU correctness"):

* per-parameter gradient cosine >= 0.99 between the gfx950 kernels and the CPU executor (fp32
  torch reference ops) for ResNet-50, BERT and Transformer, on every parameter whose gradient is
  not negligible (zero-initialised BN gammas make some branches' weight gradients exactly 0 at
  step 0; those are compared by norm instead);
* a 20-step training-loss trajectory on the GPU within 2 % of the CPU executor at every step
  (same init, same batch, same optimizer), for ResNet (SGD momentum), BERT (LAMB) and the
  Transformer (Adam).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def _resnet(dev):
    from tensorflow_k8s_amd.models.resnet import ResNet
    return ResNet(50, num_classes=100).to(dev, seed=3)


def _resnet_small(dev):
    from tensorflow_k8s_amd.models.resnet import ResNet
    return ResNet(50, stages=[1, 1, 1, 1], num_classes=100).to(dev, seed=3)


def _resnet_batch(m, dev, n=8, size=64):
    from tensorflow_k8s_amd.models.resnet import synthetic_imagenet
    x, y = synthetic_imagenet(n, "cpu", image_size=size, num_classes=100, seed=5)
    return x.to(dev), y.to(dev)


def _bert(dev):
    from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining
    c = BertConfig.tiny()
    c.hidden_dropout = c.attn_dropout = 0.0
    return BertForPreTraining(c).to(dev, seed=3)


def _transformer(dev):
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    c = TransformerConfig.tiny()
    c.dropout = c.attn_dropout = c.relu_dropout = 0.0
    return Transformer(c).to(dev, seed=3)


MODELS = {
    "resnet50": (_resnet, lambda m, d: _resnet_batch(m, d)),
    "resnet50-1111": (_resnet_small, lambda m, d: _resnet_batch(m, d)),
    "bert": (_bert, lambda m, d: tuple(t.to(d) for t in m.synthetic_batch(4, "cpu", seed=5))),
    "transformer": (_transformer, lambda m, d: tuple(t.to(d) for t in m.synthetic_batch(4, "cpu", seed=5))),
}


@pytest.mark.parametrize("which", list(MODELS))
def test_per_parameter_gradient_cosine(which):
    """resnet50: real init -- the zero-initialised residual-branch gammas (bn*_branch2c) block the
    branch gradients at step 0, so the identity/projection paths, every BN and the classifier are
    compared. resnet50-1111 (one bottleneck per stage: stem, projection + strided shortcuts, every
    kernel variant) un-zeroes those gammas so every parameter's gradient is exercised.
    (At full depth with non-zero branch gammas the stem's cosine is ~0.8 GPU-vs-CPU. That is the
    network, not the kernels: in fp32 on the CPU alone, perturbing the weights by 1e-3 relative --
    less than bf16 rounding -- drops it to 0.49 (tools/grad_parity_diag.py --perturb 1e-3,
    profiles/grad_sensitivity_r2.md): a 16-block random-init ResNet with active branches is chaotic.)"""
    mk, batch = MODELS[which]
    grads = {}
    for dev in ("cpu", "cuda"):
        m = mk(dev)
        if which != "resnet50":
            for p in m.arena.params:
                if p.name.endswith("/gamma") and float(p.master.abs().sum()) == 0.0:
                    p.master.fill_(0.5)
            m.arena.refresh_compute()
        loss, _ = m.forward_backward(*batch(m, dev))
        grads[dev] = {p.name: p.grad.detach().float().cpu().clone() for p in m.arena.params}
    gc, gg = grads["cpu"], grads["cuda"]
    norms = sorted(float(v.norm()) for v in gc.values())
    floor = 1e-3 * norms[len(norms) // 2]
    worst, checked = [], 0
    for n in gc:
        if float(gc[n].norm()) <= floor:
            assert float(gg[n].norm()) <= 10 * floor + 1e-6, (n, float(gg[n].norm()))
            continue
        checked += 1
        c = _cos(gg[n], gc[n])
        if c < 0.99:
            worst.append((n, round(c, 4)))
    assert checked >= (0.25 if which == "resnet50" else 0.9) * len(gc), (checked, len(gc))
    assert not worst, worst


def _trajectory(which, dev, steps):
    from tensorflow_k8s_amd.runtime.optimizer import LAMB, SGD, AdamW
    if which == "resnet50":
        m = _resnet_small(dev)
        b = _resnet_batch(m, dev, n=16)
        opt = SGD(m.arena, lr=0.02, momentum=0.9, weight_decay=5e-5)
    elif which == "bert":
        m = _bert(dev)
        b = MODELS["bert"][1](m, dev)
        opt = LAMB(m.arena, lr=2e-3, weight_decay=0.01)
    else:
        m = _transformer(dev)
        b = MODELS["transformer"][1](m, dev)
        opt = AdamW(m.arena, lr=1e-3, b2=0.98, eps=1e-9, weight_decay=0.0)
    out = []
    for _ in range(steps):
        loss, _ = m.forward_backward(*b)
        opt.step()
        out.append(float(loss.float().mean()))
    return out


@pytest.mark.parametrize("which", ["resnet50", "bert", "transformer"])
def test_20_step_loss_trajectory_matches_cpu(which):
    lc = _trajectory(which, "cpu", 20)
    lg = _trajectory(which, "cuda", 20)
    assert lc[-1] < lc[0], lc  # it trains
    rel = [abs(a - b) / abs(a) for a, b in zip(lc, lg)]
    assert max(rel) <= 0.02, [(i, round(a, 4), round(b, 4)) for i, (a, b) in enumerate(zip(lc, lg))]


def _fullwidth(which, seq):
    """Full-width BERT-base / Transformer-big layers (hidden 768 x 12 heads / 1024 x 16 heads, FFN
    3072 / 4096, the real vocabularies), 2 layers deep, dropout ON at the models' defaults."""
    if which == "bert-base":
        from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining
        return lambda: BertForPreTraining(BertConfig(layers=2, seq_len=seq, max_position=max(512, seq)))
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    return lambda: Transformer(TransformerConfig(enc_layers=1, dec_layers=1, src_len=seq, tgt_len=seq))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("which,seq", [("bert-base", 128), ("bert-base", 512), ("transformer-big", 256)])
def test_fullwidth_dropout_on_gradient_cosine(which, seq):
    """GPU kernels vs the fp32 CPU executor at full layer width with dropout ON: both sides draw the
    same masks (the hash RNG of salt + device key has a bit-exact CPU reference), batch 2, one step;
    every non-negligible parameter gradient has cosine >= 0.99 and the losses agree within 2 %."""
    mk = _fullwidth(which, seq)
    out = {}
    for dev in ("cpu", "cuda"):
        m = mk().to(dev, seed=3)
        assert m.training and m.rng_state is not None
        batch = tuple(t.to(dev) for t in m.synthetic_batch(2, "cpu", seed=5))
        loss, _ = m.forward_backward(*batch)
        out[dev] = (float(loss.float().mean()), {p.name: p.grad.detach().float().cpu().clone() for p in m.arena.params},
                    m.rng_state.cpu().clone())
    (lc, gc, sc), (lg, gg, sg) = out["cpu"], out["cuda"]
    assert torch.equal(sc, sg) and int(sc[0]) == 1  # same per-step key on both sides
    assert abs(lc - lg) <= 0.02 * abs(lc), (lc, lg)
    norms = sorted(float(v.norm()) for v in gc.values())
    floor = 1e-3 * norms[len(norms) // 2]
    worst, checked = [], 0
    for n in gc:
        if float(gc[n].norm()) <= floor:
            continue
        checked += 1
        c = _cos(gg[n], gc[n])
        if c < 0.99:
            worst.append((n, round(c, 4)))
    assert checked >= 0.9 * len(gc), (checked, len(gc))
    assert not worst, worst
