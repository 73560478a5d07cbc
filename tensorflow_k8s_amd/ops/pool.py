"""NHWC pooling ops (csrc/kernels/pool.hip)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._lib import lib, on_gpu


def _out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def maxpool_fwd(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1, bn=None):
    """bn = (scale, shift): pool relu(x*scale + shift) (bf16-rounded) -- the producer BatchNorm's
    apply fused into the pool, so its output is never materialized."""
    N, H, W, C = x.shape
    P, Q = _out(H, k, s, p), _out(W, k, s, p)
    if not on_gpu(x):
        if bn is not None:
            x = torch.relu(x.float() * bn[0] + bn[1]).to(torch.bfloat16)
        xn = x.float().permute(0, 3, 1, 2)
        y, idx = F.max_pool2d(xn, k, s, p, return_indices=True)
        return y.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), (idx, xn.shape)
    y = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=x.device)
    idx = torch.empty(N, P, Q, C, dtype=torch.uint8, device=x.device)
    lib().maxpool_fwd(x, y, idx, [N, H, W, C, P, Q, k, k, s, s, p, p], list(bn) if bn is not None else [])
    return y, idx


def maxpool_bwd(dy: torch.Tensor, idx, x_shape, k: int = 3, s: int = 2, p: int = 1, bnr=None) -> torch.Tensor:
    """dx of a max pool (gradients of overlapping windows accumulate). bnr (ops.norm.BNReduce, no
    second BN): also accumulate the BN-backward channel sums of the layer that produced x from the
    final dx (the ResNet stem: saves the standalone reduction's re-read of dx and y)."""
    N, H, W, C = x_shape
    if bnr is not None and bnr.y2 is not None:
        raise ValueError("maxpool_bwd BN reduce supports one BN")
    if not on_gpu(dy):
        # overlapping windows: gradients of windows sharing an argmax must ACCUMULATE
        ind, nshape = idx
        g = dy.float().permute(0, 3, 1, 2).reshape(N, C, -1)
        dx = torch.zeros(N, C, H * W).scatter_add_(2, ind.reshape(N, C, -1), g)
        dx = dx.reshape(N, C, H, W).permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
        if bnr is not None:
            bnr.reference_accumulate(dx)
        return dx
    P, Q = dy.shape[1], dy.shape[2]
    dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dy.device)
    if bnr is not None and 256 % (C // 8) != 0:
        raise ValueError("maxpool_bwd BN reduce needs (C/8) | 256")
    lib().maxpool_bwd(dy, idx, dx, [N, H, W, C, P, Q, k, k, s, s, p, p],
                      bnr.gemm_args() if bnr is not None else [], bnr.st.shards if bnr is not None else 1)
    return dx


def avgpool_fwd(x: torch.Tensor) -> torch.Tensor:
    N, H, W, C = x.shape
    if not on_gpu(x):
        return x.float().mean(dim=(1, 2)).to(torch.bfloat16)
    y = torch.empty(N, C, dtype=torch.bfloat16, device=x.device)
    lib().avgpool_fwd(x, y, N, H * W, C)
    return y


def avgpool_bwd(dy: torch.Tensor, x_shape) -> torch.Tensor:
    N, H, W, C = x_shape
    if not on_gpu(dy):
        return (dy.float()[:, None, None, :] / (H * W)).expand(N, H, W, C).to(torch.bfloat16).contiguous()
    dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dy.device)
    lib().avgpool_bwd(dy, dx, N, H * W, C)
    return dx
