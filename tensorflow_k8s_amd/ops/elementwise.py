"""Elementwise ops (csrc/kernels/misc.hip): bias+activation, activation backward, dropout, add.

Most activations are fused into GEMM epilogues (ops.gemm act=...); these standalone passes cover
the remaining producers. act: None | "relu" | "gelu" (tanh form, as TF's gelu(approximate=True)) | "tanh".
"""
from __future__ import annotations

import contextlib

import torch

from ._lib import lib, on_gpu
from .gemm import ACT, act_grad_ref, act_ref

_M64 = (1 << 64) - 1


def _s64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >> 63 else v


def _shr(x: torch.Tensor, k: int) -> torch.Tensor:
    return (x >> k) & ((1 << (64 - k)) - 1)


def hash_u32(seed, idx: torch.Tensor) -> torch.Tensor:
    """Bit-exact torch (int64) copy of common.h hash_u32(seed, idx); seed: int or int64 tensor."""
    sd = seed if torch.is_tensor(seed) else torch.tensor(_s64(int(seed)), dtype=torch.int64)
    x = (idx * _s64(0x9E3779B97F4A7C15)) ^ (sd + _s64(0xD1B54A32D192ED03))
    x = x ^ _shr(x, 31)
    x = x * _s64(0xBF58476D1CE4E5B9)
    x = x ^ _shr(x, 27)
    x = x * _s64(0x94D049BB133111EB)
    x = x ^ _shr(x, 33)
    return x & 0xFFFFFFFF


def u01(h: torch.Tensor) -> torch.Tensor:
    return (h >> 8).float() * (1.0 / 16777216.0)


def hash32(x):
    """Bit-exact copy of common.h hash32 (lowbias32) on int64 tensors holding uint32 (or ints)."""
    m = 0xFFFFFFFF
    x = x & m
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & m
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & m
    return x ^ (x >> 16)


def drop_seed32(seed: int) -> int:
    """common.h drop_seed32: the 64-bit dropout seed folded to the 32-bit stream seed."""
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    return int(hash32((s & 0xFFFFFFFF) ^ int(hash32(((s >> 32) ^ 0x9E3779B9) & 0xFFFFFFFF))))


# ------------------------------------------------------------------ per-step device RNG key
# Dropout seed = host per-site salt + a per-step key that lives ON THE DEVICE in the model's rng state
# (int64 [counter, key]). rng_advance() steps it inside the training step, so a replayed hipGraph
# draws fresh masks every step; rng_key() registers the state for every dropout-capable launch
# (GEMM epilogues, dropout, LayerNorm-backward dropout, attention) while a step runs.
_KEY: torch.Tensor | None = None


@contextlib.contextmanager
def rng_key(state: torch.Tensor | None):
    global _KEY
    prev, _KEY = _KEY, state
    gpu = state is not None and state.is_cuda
    if gpu:
        lib().set_rng_key(state)
    try:
        yield
    finally:
        _KEY = prev
        if gpu:
            lib().set_rng_key(prev if prev is not None and prev.is_cuda else None)


def rng_advance(state: torch.Tensor, stream: int = 0) -> None:
    """counter += 1; key = splitmix64(counter ^ stream) (misc.hip rng_advance_kernel)."""
    if state.is_cuda:
        lib().rng_advance(state, int(stream))
        return
    m = _M64
    c = (int(state[0]) + 1) & m
    z = ((c ^ (int(stream) & m)) + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    state[0] = _s64(c)
    state[1] = _s64(z ^ (z >> 31))


def eff_seed(salt: int) -> int:
    """The seed a kernel launched now uses for this salt (host reference of common.h eff_seed)."""
    if _KEY is None:
        return int(salt)
    return _s64(int(salt) + int(_KEY[1]))


def drop_thr8(p: float) -> int:
    """common.h drop_thr8: the 8-bit drop threshold round(256 p), in the kernels' float arithmetic."""
    import numpy as np
    t = int(np.float32(p) * np.float32(256.0) + np.float32(0.5))
    return max(0, min(255, t))


def check_rate(p: float) -> float:
    """Dropout rates the 8-bit mask threshold represents: the kernels drop an element iff a hash
    byte < thr = round(256 p), so the EFFECTIVE rate is thr / 256 (p = 0.1 runs at 0.1016,
    p = 0.3 at 0.3008; the 256 / (256 - thr) keep scale keeps it unbiased). Rejected: 0 < p < 1/512
    (thr = 0: nothing would be dropped) and p > 255.5/256 (thr caps at 255: 1/256 of the elements
    would survive, scaled by 256, instead of all being dropped). Returns p."""
    p = float(p)
    if p < 0.0 or p >= 1.0:
        raise ValueError(f"dropout rate must be in [0, 1), got {p}")
    if p > 0.0 and drop_thr8(p) == 0:
        raise ValueError(f"dropout rate {p} < 1/512 rounds to no dropout in the 8-bit mask; use 0 or >= 1/512")
    if p > 255.5 / 256.0:
        raise ValueError(f"dropout rate {p} > 255.5/256 is not representable by the 8-bit mask")
    return p


def effective_rate(p: float) -> float:
    """The drop probability the kernels actually apply for nominal rate p (thr / 256)."""
    return drop_thr8(p) / 256.0


def keep_scale(p: float) -> float:
    """Inverse keep probability of the quantized mask, 256 / (256 - thr) (common.h drop_scale8)."""
    import numpy as np
    return float(np.float32(256.0) / np.float32(256 - drop_thr8(p)))


def dropout_keep(seed: int, n: int, p: float) -> torch.Tensor:
    """Keep-mask of the dropout kernel / fused GEMM dropout over a contiguous tensor of n elements:
    element i kept iff byte (i & 3) of hash32(s32 ^ (i >> 2)) >= round(256 p) (common.h drop_keep1)."""
    idx = torch.arange(n, dtype=torch.int64)
    h = hash32(drop_seed32(seed) ^ ((idx >> 2) & 0xFFFFFFFF))
    return ((h >> (8 * (idx & 3))) & 0xFF) >= drop_thr8(p)


def act_fwd(x: torch.Tensor, act: str | None, bias: torch.Tensor | None = None) -> torch.Tensor:
    if not on_gpu(x):
        v = x.float() + (bias.float() if bias is not None else 0.0)
        return act_ref(v, act).to(torch.bfloat16)
    y = torch.empty_like(x)
    lib().act_fwd(x, bias, x.shape[-1], y, ACT[act])
    return y


def act_bwd(dy: torch.Tensor, x: torch.Tensor, act: str | None) -> torch.Tensor:
    """dx = dy * act'(x). For relu, x may be the pre- or post-activation (same sign test)."""
    if not on_gpu(dy):
        return (dy.float() * act_grad_ref(x, act)).to(torch.bfloat16)
    dx = torch.empty_like(dy)
    lib().act_bwd(dy, x, dx, ACT[act])
    return dx


def dropout(x: torch.Tensor, p: float, seed: int) -> torch.Tensor:
    """Inverted dropout; the mask is a hash of (seed, index), so backward = dropout(dy, p, seed)."""
    if p <= 0.0:
        return x
    check_rate(p)
    if not on_gpu(x):
        keep = dropout_keep(eff_seed(seed), x.numel(), p).reshape(x.shape)
        return (x.float() * keep * keep_scale(p)).to(torch.bfloat16)
    y = torch.empty_like(x)
    lib().dropout(x, y, p, int(seed))
    return y


def add(a: torch.Tensor, b: torch.Tensor, alpha: float = 1.0, beta: float = 1.0) -> torch.Tensor:
    if not on_gpu(a):
        return (alpha * a.float() + beta * b.float()).to(torch.bfloat16)
    y = torch.empty_like(a)
    lib().add(a, b, y, alpha, beta)
    return y
