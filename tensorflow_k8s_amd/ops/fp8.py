"""MX-fp8 linear layers (csrc/kernels/fp8.hip): OCP e4m3 values with one e8m0 (power-of-two)
scale per 32 K-elements of each row, multiplied by gfx950's block-scaled MFMA
(v_mfma_scale_f32_16x16x128_f8f6f4, 2x the bf16 MFMA rate).

Used for the forward GEMMs of the transformer models when ``fp8=True`` (activations and weights
are quantized on the fly; the f32 master weights, the optimizer and the backward pass stay in
bf16/f32). The CPU path is the exact dequantized reference of the same quantization.
"""
from __future__ import annotations

import torch

from ._lib import lib, on_gpu
from .gemm import ACT, act_ref

E4M3_MAX = 448.0
MX_BLOCK = 32


def _scale_exponent(amax: torch.Tensor) -> torch.Tensor:
    e = torch.ceil(torch.log2(amax / E4M3_MAX))
    e = torch.where(amax > 0, e, torch.full_like(e, -127.0))
    return e.clamp(-127, 127)


def mx_quantize(x: torch.Tensor):
    """bf16 [rows, K] (K % 32 == 0) -> (q uint8 e4m3 [rows, K], s uint8 e8m0 [rows, K/32])."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    rows = x2.shape[0]
    if K % MX_BLOCK:
        raise ValueError(f"MX quantization needs K % 32 == 0, got {K}")
    if not on_gpu(x):
        xb = x2.float().view(rows, K // MX_BLOCK, MX_BLOCK)
        e = _scale_exponent(xb.abs().amax(-1))
        v = (xb * torch.exp2(-e)[..., None]).clamp(-E4M3_MAX, E4M3_MAX)
        q = v.to(torch.float8_e4m3fn).view(torch.uint8).reshape(rows, K)
        return q, (e + 127).to(torch.uint8)
    q = torch.empty(rows, K, dtype=torch.uint8, device=x.device)
    s = torch.empty(rows, K // MX_BLOCK, dtype=torch.uint8, device=x.device)
    lib().mx_quant(x2, q, s, rows, K)
    return q, s


def mx_dequantize(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    rows, K = q.shape
    v = q.cpu().view(torch.float8_e4m3fn).float().view(rows, K // MX_BLOCK, MX_BLOCK)
    return (v * torch.exp2(s.cpu().float() - 127)[..., None]).reshape(rows, K)


def linear_fwd_mx(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
                  resid: torch.Tensor | None = None, aux: torch.Tensor | None = None, drop_p: float = 0.0,
                  drop_seed: int = 0, wq=None) -> torch.Tensor:
    """y[M,N] = dropout(act(MX(x) @ MX(w)^T + bias)) (+ resid), bf16 out. wq: pre-quantized weight."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M, N = x2.shape[0], w.shape[0]
    if K % 128:
        raise ValueError(f"MX-fp8 GEMM needs K % 128 == 0, got {K}")
    xq, xs = mx_quantize(x2)
    wq_, ws_ = wq if wq is not None else mx_quantize(w)
    if not on_gpu(x):
        y = mx_dequantize(xq, xs) @ mx_dequantize(wq_, ws_).t()
        if bias is not None:
            y = y + bias.float()
        if aux is not None:
            aux.view(-1, N).copy_(y)
        y = act_ref(y, act)
        if drop_p > 0:
            from .elementwise import dropout_keep
            y = y * dropout_keep(drop_seed, y.numel(), drop_p).reshape(y.shape) / (1 - drop_p)
        y = y.to(torch.bfloat16)
        if resid is not None:
            y = (y.float() + resid.reshape(-1, N).float()).to(torch.bfloat16)
        return y
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    lib().gemm_mxfp8(xq, xs, wq_, ws_, y, M, N, K, bias, resid.reshape(-1, N) if resid is not None else None,
                     ACT[act], aux, drop_p, drop_seed)
    return y
