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


def resnet_loss(model, x_nhwc, labels, smoothing):
    """Returns (loss, {param_name: leaf tensor}) with leaves in storage layout (f32)."""
    leaves = {p.name: p.master.detach().clone().float().requires_grad_(True) for p in model.arena.params}

    def conv(layer, h):
        w = leaves[layer.w.name].permute(0, 3, 1, 2)
        return F.conv2d(h, w, stride=layer.stride, padding=layer.pad)

    def bn(layer, h):
        return _bn(h, leaves[layer.gamma.name], leaves[layer.beta.name], layer.eps)

    h = x_nhwc.float().permute(0, 3, 1, 2)
    h = F.relu(bn(model.bn1, conv(model.conv1, h)))
    h = F.max_pool2d(h, 3, 2, 1)
    for b in model.blocks:
        o = F.relu(bn(b.bn1, conv(b.conv1, h)))
        o = F.relu(bn(b.bn2, conv(b.conv2, o)))
        o = bn(b.bn3, conv(b.conv3, o))
        sc = bn(b.bn_sc, conv(b.conv_sc, h)) if b.proj else h
        h = F.relu(o + sc)
    f = h.mean(dim=(2, 3))
    logits = f @ leaves[model.fc.w.name].t() + leaves[model.fc.b.name]
    loss = F.cross_entropy(logits, labels.long(), label_smoothing=smoothing)
    return loss, leaves
