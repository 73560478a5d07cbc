"""Plain-torch fp32 autograd references of the tfk models, driven by the SAME arena weights.
Used as the numerics oracle for the executor's hand-written backward passes."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _bn(x, gamma, beta, eps):
    # x NCHW, training-mode batch statistics (biased variance)
    mean = x.mean(dim=(0, 2, 3), keepdim=True)
    var = x.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    return (x - mean) / torch.sqrt(var + eps) * gamma[None, :, None, None] + beta[None, :, None, None]


class _Round(torch.autograd.Function):
    """bf16 storage of an activation AND of its gradient, as the executor keeps them."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def resnet_loss(model, x_nhwc, labels, smoothing, emulate_bf16=False):
    """Returns (loss, {param_name: leaf tensor}) with leaves in storage layout (f32). With
    emulate_bf16 the activations/weights are rounded to bf16 where the executor stores them:
    random-init deep ResNets are chaotic enough that pure-fp32 and bf16 forwards drift apart by
    ~50% at the last stage (measured), so exact-ish comparisons need the emulated reference."""
    leaves = {p.name: p.master.detach().clone().float().requires_grad_(True) for p in model.arena.params}
    rd = _Round.apply if emulate_bf16 else (lambda t: t)

    def conv(layer, h):
        w = leaves[layer.w.name].permute(0, 3, 1, 2)
        if emulate_bf16:
            w = w.to(torch.bfloat16).float()
        return rd(F.conv2d(h, w, stride=layer.stride, padding=layer.pad))

    def bn(layer, h):
        return _bn(h, leaves[layer.gamma.name], leaves[layer.beta.name], layer.eps)

    h = x_nhwc.float().permute(0, 3, 1, 2)
    h = rd(F.relu(bn(model.bn1, conv(model.conv1, h))))
    h = F.max_pool2d(h, 3, 2, 1)
    for b in model.blocks:
        o = rd(F.relu(bn(b.bn1, conv(b.conv1, h))))
        o = rd(F.relu(bn(b.bn2, conv(b.conv2, o))))
        o = bn(b.bn3, conv(b.conv3, o))
        sc = bn(b.bn_sc, conv(b.conv_sc, h)) if b.proj else h
        h = rd(F.relu(o + sc))
    f = rd(h.mean(dim=(2, 3)))
    wfc = leaves[model.fc.w.name]
    if emulate_bf16:
        wfc = wfc.to(torch.bfloat16).float()
    logits = rd(f @ wfc.t() + leaves[model.fc.b.name])
    loss = F.cross_entropy(logits, labels.long(), label_smoothing=smoothing)
    return loss, leaves
