"""Out-of-bounds / unwritten-output detection for the hand-written kernels (SURVEY §5.2 "race
detection" on the GPU side, where no GPU sanitizer is available on this pool).

Every device buffer an op allocates (torch.empty / empty_like, patched for the duration of the
call) is placed inside a larger allocation: the payload is poisoned with NaN and flanked by
GUARD-element canary bands of a distinct NaN bit pattern. After the op:
  * every canary band must be bit-identical (no write past either end of any buffer -- outputs,
    workspaces, split-K slabs, statistics);
  * every returned output must hold no NaN (every element was written, incl. ragged tails and
    padding columns a kernel promises to write).
Caller-provided outputs (weight-gradient accumulators, dq/dk/dv views) are guarded the same way
by the test itself. Shapes are ragged on purpose: partial tiles in M, N and K, odd image sizes,
padded vocabularies, key padding and causal masks.
"""
import math

import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops import loss as LS
from tensorflow_k8s_amd.ops import norm as BN
from tensorflow_k8s_amd.ops import transformer as T
from tensorflow_k8s_amd.ops._lib import lib

pytestmark = pytest.mark.gpu

GUARD = 1 << 16  # elements per canary band
_CANARY = {torch.bfloat16: (torch.int16, 0x7FA5), torch.float32: (torch.int32, 0x7FA5A5A5)}
_POISON = {torch.bfloat16: (torch.int16, 0x7FC0), torch.float32: (torch.int32, 0x7FC00000)}


class Guarded:
    """Guard-banded allocator for cuda bf16/f32 tensors."""

    def __init__(self):
        self.bufs = []
        self._empty = torch.empty
        self._empty_like = torch.empty_like

    def alloc(self, shape, dtype):
        n = math.prod(shape)
        it, cv = _CANARY[dtype]
        buf = self._empty(n + 2 * GUARD, dtype=dtype, device="cuda")
        buf.view(it).fill_(cv)
        _, pv = _POISON[dtype]
        buf[GUARD:GUARD + n].view(it).fill_(pv)
        self.bufs.append((buf, n, dtype))
        return buf[GUARD:GUARD + n].view(shape)

    def empty(self, *size, dtype=None, device=None, **kw):
        shape = tuple(size[0]) if len(size) == 1 and isinstance(size[0], (tuple, list, torch.Size)) else tuple(size)
        dt = dtype or torch.get_default_dtype()
        if device is not None and torch.device(device).type == "cuda" and dt in _CANARY and not kw:
            return self.alloc(shape, dt)
        return self._empty(*size, dtype=dtype, device=device, **kw)

    def empty_like(self, x, **kw):
        if x.is_cuda and x.dtype in _CANARY and not kw:
            return self.alloc(tuple(x.shape), x.dtype)
        return self._empty_like(x, **kw)

    def __enter__(self):
        torch.empty, torch.empty_like = self.empty, self.empty_like
        return self

    def __exit__(self, *a):
        torch.empty, torch.empty_like = self._empty, self._empty_like

    def check(self):
        torch.cuda.synchronize()
        for i, (buf, n, dt) in enumerate(self.bufs):
            it, cv = _CANARY[dt]
            raw = buf.view(it)
            lo, hi = raw[:GUARD], raw[GUARD + n:]
            bad_lo = int((lo != cv).sum())
            bad_hi = int((hi != cv).sum())
            assert bad_lo == 0 and bad_hi == 0, f"buffer {i} ({dt}, {n} elems): {bad_lo} writes below, {bad_hi} above"


def no_nan(*ts):
    for i, t in enumerate(ts):
        assert not torch.isnan(t.float()).any(), f"output {i} has unwritten (NaN-poisoned) elements"


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).cuda()


@pytest.mark.parametrize("M,N,K", [(1000, 520, 72), (300, 264, 200), (33000, 200, 136), (129, 136, 64)])
def test_gemm_guard(M, N, K):
    x, w, dy = bf(M, K, seed=1), bf(N, K, scale=0.05, seed=2), bf(M, N, seed=3)
    with Guarded() as g:
        y = G.linear_fwd(x, w, act="relu")
        dx = G.linear_dgrad(dy, w)
        gw = g.alloc((N, K), torch.float32)
        G.linear_wgrad(dy, x, gw)
    g.check()
    no_nan(y, dx, gw)


@pytest.mark.parametrize("cfg", [(3, 9, 11, 128, 200, 3, 3, 2, 1), (2, 14, 13, 64, 128, 1, 1, 1, 0),
                                 (2, 15, 15, 64, 64, 3, 3, 1, 1), (2, 31, 29, 8, 64, 7, 7, 2, 3)])
def test_conv_guard(cfg):
    N, H, W, C, K, R, S, st, pd = cfg
    geo = G.ConvGeom(N, H, W, C, K, R, S, st, st, pd, pd)
    x = bf(N, H, W, C, seed=1)
    w = bf(K, R, S, C, scale=0.05, seed=2)
    dy = bf(N, geo.P, geo.Q, K, seed=3)
    with Guarded() as g:
        stats = g.alloc((8 * 2 * K,), torch.float32)
        stats.zero_()
        y = G.conv_fwd(x, w, geo, stats, 8)
        dx = G.conv_dgrad(dy, w, geo) if C % 8 == 0 and C >= 64 else None
        gw = g.alloc((K, R, S, C), torch.float32)
        G.conv_wgrad(dy, x, geo, gw)
    g.check()
    no_nan(y, gw, stats, *([dx] if dx is not None else []))


def test_conv_dgrad_bnr_guard():
    """1x1 dgrad with the fused BN-backward reduction and an identity-shortcut residual."""
    N, H, W, C, K = 2, 13, 15, 128, 64
    geo = G.ConvGeom(N, H, W, C, K, 1, 1)
    w = bf(K, 1, 1, C, scale=0.05, seed=2)
    dy = bf(N, H, W, K, seed=3)
    y, a, r = bf(N, H, W, C, seed=5), bf(N, H, W, C, seed=6), bf(N, H, W, C, seed=7)
    with Guarded() as g:
        st = BN.BNState(C, "cuda")
        st.mean.copy_(torch.randn(C) * 0.1)
        st.invstd.copy_(torch.rand(C) + 0.5)
        dx = G.conv_dgrad(dy, w, geo, resid=r, bnr=BN.BNReduce(y, st, a=a))
    g.check()
    no_nan(dx, st.sums)


@pytest.mark.parametrize("causal,padded", [(False, True), (True, False), (True, True)])
def test_attention_guard(causal, padded):
    B, H, S = 3, 4, 77
    D = T.HEAD_DIM
    qkv = bf(B * S, 3 * H * D, scale=0.5, seed=1)
    kv_len = torch.tensor([77, 40, 13], dtype=torch.int32, device="cuda") if padded else None
    sp = T.AttnSpec(B, H, S, S, (qkv, 0), (qkv, H * D), (qkv, 2 * H * D), kv_len=kv_len, causal=causal)
    dout = bf(B * S, H * D, seed=2)
    with Guarded() as g:
        out, lse = T.attention_fwd(sp)
        dqkv = g.alloc((B * S, 3 * H * D), torch.bfloat16)
        T.attention_bwd(sp, out, dout, lse, (dqkv, 0), (dqkv, H * D), (dqkv, 2 * H * D))
    g.check()
    if padded:
        # rows of fully padded keys have no defined lse; outputs and grads must still be written
        no_nan(out, dqkv)
    else:
        no_nan(out, lse, dqkv)


@pytest.mark.parametrize("B,V,ld", [(37, 1000, 1024), (5, 33708, 33728), (9, 50000, 50048), (3, 130, 130)])
def test_xent_guard(B, V, ld):
    logits = bf(B, ld, scale=3.0, seed=1)
    labels = torch.randint(0, V, (B,), dtype=torch.int32, device="cuda")
    labels[0] = -100
    with Guarded() as g:
        loss, d, corr = LS.softmax_xent(logits, labels, smoothing=0.1, scale=0.5, want_correct=True, V=V)
    g.check()
    no_nan(loss, d, corr)
    if ld > V:
        assert float(d[:, V:].float().abs().max()) == 0.0


def test_layernorm_guard():
    M, W = 333, 768
    x = bf(M, W, seed=1)
    gamma = torch.randn(W, device="cuda")
    beta = torch.randn(W, device="cuda")
    dy = bf(M, W, seed=2)
    with Guarded() as g:
        y, mean, rstd = T.layernorm_fwd(x, gamma, beta)
        dg = g.alloc((W,), torch.float32)
        db = g.alloc((W,), torch.float32)
        dx = T.layernorm_bwd(dy, x, gamma, mean, rstd, dg, db)
    g.check()
    no_nan(y, mean, rstd, dx, dg, db)


def test_guard_detects_an_overrun():
    """Self-test: a deliberate one-element overrun into the upper band is reported."""
    with Guarded() as g:
        t = torch.empty(100, dtype=torch.float32, device="cuda")
    t.fill_(0.0)
    full = g.bufs[0][0]
    full[GUARD + 100] = 1.0
    with pytest.raises(AssertionError, match="1 above"):
        g.check()
    lib()  # native library loaded (ops above ran on it)
