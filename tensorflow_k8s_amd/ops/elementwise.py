"""Elementwise ops (csrc/kernels/misc.hip): bias+activation, activation backward, dropout, add.

Most activations are fused into GEMM epilogues (ops.gemm act=...); these standalone passes cover
the remaining producers. act: None | "relu" | "gelu" (tanh form, as TF's gelu(approximate=True)).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import lib, on_gpu

ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2}


def act_fwd(x: torch.Tensor, act: str | None, bias: torch.Tensor | None = None) -> torch.Tensor:
    if not on_gpu(x):
        v = x.float() + (bias.float() if bias is not None else 0.0)
        if ACT[act] == 1:
            v = torch.relu(v)
        elif ACT[act] == 2:
            v = F.gelu(v, approximate="tanh")
        return v.to(torch.bfloat16)
    y = torch.empty_like(x)
    lib().act_fwd(x, bias, x.shape[-1], y, ACT[act])
    return y


def act_bwd(dy: torch.Tensor, x: torch.Tensor, act: str | None) -> torch.Tensor:
    """dx = dy * act'(x). For relu, x may be the pre- or post-activation (same sign test)."""
    if not on_gpu(dy):
        g = dy.float()
        if ACT[act] == 1:
            g = g * (x.float() > 0)
        elif ACT[act] == 2:
            xf = x.float().requires_grad_(True)
            with torch.enable_grad():
                (gx,) = torch.autograd.grad(F.gelu(xf, approximate="tanh"), xf, g)
            g = gx
        return g.to(torch.bfloat16)
    dx = torch.empty_like(dy)
    lib().act_bwd(dy, x, dx, ACT[act])
    return dx


def dropout(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """Inverted dropout; the mask is a hash of (seed, index), so backward = dropout(dy, p, seed)."""
    if p <= 0.0:
        return x
    if not on_gpu(x):
        g = torch.Generator().manual_seed(int(seed))
        keep = torch.rand(x.shape, generator=g) >= p
        return (x.float() * keep / (1 - p)).to(torch.bfloat16)
    y = torch.empty_like(x)
    lib().dropout(x, y, p, int(seed))
    return y


def add(a: torch.Tensor, b: torch.Tensor, alpha: float = 1.0, beta: float = 1.0) -> torch.Tensor:
    if not on_gpu(a):
        return (alpha * a.float() + beta * b.float()).to(torch.bfloat16)
    y = torch.empty_like(a)
    lib().add(a, b, y, alpha, beta)
    return y
