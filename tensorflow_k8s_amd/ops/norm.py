"""Training-mode BatchNorm for NHWC bf16 activations (csrc/kernels/bn.hip).

Forward statistics come from the producing conv's GEMM epilogue (``stats`` buffer), so the
forward is finalize + one fused apply pass; the projection-shortcut BN can be folded into the
residual add of the same pass (dual form). Backward is reduce -> finalize -> apply.
"""
from __future__ import annotations


import os

import torch

from ._lib import lib, on_gpu

# f32 atomic shards of the BN statistics / backward sums (GEMM epilogues spread their per-block
# partial sums over SHARDS copies; finalize kernels reduce them). Measured
# (ResNet-50 bs256 step, same box): 8 -> 25.21, 12 -> 25.33, 16 -> 25.15-25.19, 32 -> 25.25-25.41,
# 64 -> 25.70 ms -- the finalize kernels sit on the critical path and read every shard
SHARDS = 16
# Finalize folded into the apply passes (bn.hip bn_apply_fin / bn_bwd_apply_fin) for pooled states:
# no separate finalize launch between a conv and its BN pass. Opt-in (TFK_BN_FUSED_FIN=1): measured
# SLOWER in the captured ResNet-50 step (21.57 / 21.60 vs 21.31 / 21.36 ms, profiles/perf_log_r6.md) --
# the per-block finalize prologue and the 64-channel slice layout cost more than the launches saved.
FUSED_FIN = os.environ.get("TFK_BN_FUSED_FIN", "0") == "1"


class BNState:
    """Per-BN-layer device state: stats accumulators and the per-step saved statistics.
    acc: optional flat f32 view [shards*5*C] to hold stats + sums (a BNPool's slice)."""

    def __init__(self, C: int, device, shards: int = SHARDS, acc: torch.Tensor | None = None):
        self.C = C
        self.shards = shards if torch.device(device).type == "cuda" else 1
        n2, n3 = self.shards * 2 * C, self.shards * 3 * C
        if acc is None:
            acc = torch.zeros(n2 + n3, dtype=torch.float32, device=device)
        self.stats = acc[:n2]
        self.sums = acc[n2:n2 + n3]
        self.pooled = False  # a BNPool zeroes the accumulators once per step (the fused kernels need it)
        self.fin = None      # deferred forward finalize (gamma, beta, eps, momentum, run_mean, run_var)
        self.mean = torch.zeros(C, dtype=torch.float32, device=device)
        self.invstd = torch.ones(C, dtype=torch.float32, device=device)
        self.scale = torch.ones(C, dtype=torch.float32, device=device)
        self.shift = torch.zeros(C, dtype=torch.float32, device=device)
        self.coef = torch.zeros(3 * C, dtype=torch.float32, device=device)


class BNPool:
    """The accumulators (stats + backward sums) of a model's BN layers in ONE flat buffer, zeroed by
    one kernel at the start of each training step -- the finalize-in-apply kernels read the shards
    from every block of a layer's apply pass, so they cannot zero them themselves."""

    def __init__(self, Cs: list[int], device, shards: int = SHARDS):
        self.device = torch.device(device)
        shards = shards if self.device.type == "cuda" else 1
        sizes = [shards * 5 * C for C in Cs]
        self.buf = torch.zeros(sum(sizes), dtype=torch.float32, device=device)
        self.states, o = [], 0
        for C, n in zip(Cs, sizes):
            st = BNState(C, device, shards, acc=self.buf[o:o + n])
            st.pooled = True
            self.states.append(st)
            o += n

    def zero(self) -> None:
        """Zero every accumulator (only the fused kernels need it: the separate finalize kernels
        zero the shards they read)."""
        if not FUSED_FIN:
            return
        if on_gpu(self.buf):
            lib().bn_zero(self.buf)
        else:
            self.buf.zero_()


def _fused(st: BNState) -> bool:
    return FUSED_FIN and st.pooled and on_gpu(st.stats) and bool(lib().bn_fin_ok(st.C, st.shards))


def bn_finalize(st: BNState, count: float, gamma, beta, eps, momentum, run_mean, run_var, defer: bool = False) -> None:
    """defer (pooled GPU states): leave the finalize to the next bn_apply on st, which folds it into
    its pass (bn_apply_fin); count is then that pass's row count."""
    C = st.C
    if defer and _fused(st):
        st.fin = (gamma, beta, eps, momentum, run_mean, run_var)
        return
    if not on_gpu(st.stats):
        s = st.stats.view(st.shards, 2, C).sum(0)
        mean = s[0] / count
        var = (s[1] / count - mean * mean).clamp_min(0)
        inv = torch.rsqrt(var + eps)
        st.mean.copy_(mean); st.invstd.copy_(inv)
        st.scale.copy_(gamma * inv); st.shift.copy_(beta - mean * gamma * inv)
        if run_mean is not None:
            unb = var * count / max(count - 1.0, 1.0)
            run_mean.mul_(1 - momentum).add_(momentum * mean)
            run_var.mul_(1 - momentum).add_(momentum * unb)
        st.stats.zero_()
        return
    lib().bn_finalize(st.stats, st.shards, C, float(count), gamma, beta, eps, momentum, run_mean, run_var, st.mean,
                      st.invstd, st.scale, st.shift)


def bn_stats(y: torch.Tensor, st: BNState) -> None:
    """Accumulate batch statistics of y (for producers without a fused-stats epilogue)."""
    C = st.C
    if not on_gpu(y):
        yf = y.float().reshape(-1, C)
        v = st.stats.view(st.shards, 2, C)
        v[0, 0] += yf.sum(0); v[0, 1] += (yf * yf).sum(0)
        return
    lib().bn_stats(y, y.numel() // C, C, st.stats, st.shards)


def pack_relu_mask(a: torch.Tensor) -> torch.Tensor:
    """Relu bitmask of a (numel % 8 == 0): uint8 [numel/8], bit e of byte i = a[8i+e] > 0 -- the
    layout bn_apply(mask=True) writes and the BN-backward kernels / GEMM epilogue read."""
    bits = (a.reshape(-1, 8) > 0).to(torch.uint8)
    w = torch.tensor([1, 2, 4, 8, 16, 32, 64, 128], dtype=torch.uint8, device=a.device)
    return (bits * w).sum(1, dtype=torch.uint8)


def unpack_relu_mask(mask: torch.Tensor, shape) -> torch.Tensor:
    """bool tensor of `shape` from a packed relu bitmask."""
    sh = torch.arange(8, dtype=torch.uint8, device=mask.device)
    return ((mask.reshape(-1, 1) >> sh) & 1).bool().reshape(shape)


def _mask_of(a, shape) -> torch.Tensor:
    """bool relu mask from a (bf16 post-activation tensor or packed bitmask)."""
    if a.dtype == torch.uint8:
        return unpack_relu_mask(a, shape)
    return a.float().reshape(shape) > 0


def bn_apply(y, st: BNState, relu: bool, r=None, rst: BNState | None = None, out=None, mask: bool = False):
    """a = relu?(y*scale + shift [+ r | + r*rscale + rshift]).

    mask=True (relu only): also return the packed relu bitmask of a (pack_relu_mask), so the
    backward reads 1 bit per element instead of a itself: returns (a, mask)."""
    C = st.C
    if mask and not relu:
        raise ValueError("bn_apply: mask=True needs relu")
    if not on_gpu(y):
        o = y.float() * st.scale + st.shift
        if r is not None:
            o = o + (r.float() * rst.scale + rst.shift if rst is not None else r.float())
        if relu:
            o = torch.relu(o)
        o = o.to(torch.bfloat16)
        if out is not None:
            out.copy_(o)
            o = out
        return (o, pack_relu_mask(o)) if mask else o
    out = out if out is not None else torch.empty_like(y)
    mk = torch.empty(y.numel() // 8, dtype=torch.uint8, device=y.device) if mask else None
    if st.fin is not None or (rst is not None and rst.fin is not None):
        # the deferred finalize(s) of st (and the shortcut BN rst) run inside this pass
        def spec(b: BNState):
            if b.fin is None:
                return [None] * 7 + [b.scale, b.shift], 0.0, 0.0, b.shards
            gamma, beta, eps, momentum, rm, rv = b.fin
            return [b.stats, gamma, beta, rm, rv, b.mean, b.invstd, b.scale, b.shift], eps, momentum, b.shards
        f, e, m, sh = spec(st)
        f2, e2, m2, sh2 = spec(rst) if rst is not None else ([], 0.0, 0.0, 0)
        lib().bn_apply_fin(y, f, e, m, sh, r, f2, e2, m2, sh2, relu, out, y.numel() // C, C, mk)
        st.fin = None
        if rst is not None:
            rst.fin = None
        return (out, mk) if mask else out
    lib().bn_apply(y, st.scale, st.shift, r, rst.scale if rst is not None else None,
                   rst.shift if rst is not None else None, relu, out, y.numel() // C, C, mk)
    return (out, mk) if mask else out


class BNReduce:
    """Spec for fusing a BN-backward reduction into the epilogue of the GEMM that produces dA
    (dz = dA * mask; sums into st.sums). mask: `a > 0` if a is given (a: the bf16 activation or its
    packed relu bitmask), else `y*scale+shift > 0` when relu, else 1. y2/st2: projection-shortcut
    BN sharing the same dz. premask: the GEMM stores dz instead of dA (the BN backward is dA's only
    consumer: it then reads no mask, and an identity shortcut's gradient IS dz -- no second output)."""

    def __init__(self, y, st: BNState, a=None, relu: bool = True, y2=None, st2: BNState | None = None,
                 premask: bool = False):
        self.y, self.st, self.a, self.relu, self.y2, self.st2 = y, st, a, relu, y2, st2
        self.premask = premask

    def gemm_args(self):
        st, st2 = self.st, self.st2
        if self.a is not None and self.a.dtype != torch.uint8:
            self.a = pack_relu_mask(self.a)  # the epilogue reads the packed mask only
        return [self.y, self.a, st.mean, st.invstd, st.scale if (self.relu and self.a is None) else None,
                st.shift if (self.relu and self.a is None) else None, self.y2, st2.mean if st2 else None,
                st2.invstd if st2 else None, st.sums]

    def reference_accumulate(self, dA: torch.Tensor) -> torch.Tensor:
        """CPU oracle of the fused reduction (shard 0 of st.sums). Returns dz (f32 [rows, C])."""
        C = self.st.C
        dz = dA.float().reshape(-1, C)
        y = self.y.float().reshape(-1, C)
        if self.a is not None:
            dz = dz * _mask_of(self.a, (-1, C))
        elif self.relu:
            dz = dz * ((y * self.st.scale + self.st.shift) > 0)
        v = self.st.sums.view(self.st.shards, 3, C)
        v[0, 0] += dz.sum(0)
        v[0, 1] += (dz * (y - self.st.mean) * self.st.invstd).sum(0)
        if self.y2 is not None:
            y2 = self.y2.float().reshape(-1, C)
            v[0, 2] += (dz * (y2 - self.st2.mean) * self.st2.invstd).sum(0)
        return dz


def bn_backward(da, a, y, st: BNState, gamma, dgamma, dbeta, count: float, y2=None, st2: BNState | None = None,
                gamma2=None, dgamma2=None, dbeta2=None, want_dres: bool = False, relu_from_y: bool = False,
                reduced: bool = False, premasked: bool = False):
    """Backward of a = relu?(bn(y) [+ bn2(y2) | + r]).

    a: post-activation output (bf16, or its packed relu bitmask) used for the relu mask (None -> no
    relu, unless relu_from_y: the mask
    is recomputed as y*scale+shift > 0, valid when there is no residual input). reduced: the
    per-channel sums were already accumulated into st.sums by the producer's GEMM epilogue
    (BNReduce). premasked: da already is dz (BNReduce(premask=True) producer): no mask is read
    and dres is da itself. Returns (dy, dy2, dres). Writes dgamma/dbeta (and the second BN's)."""
    C = st.C
    if premasked:
        if not reduced:
            raise ValueError("bn_backward: premasked da comes from a fused-reduce producer (reduced=True)")
        a, relu_from_y = None, False
    if not on_gpu(da):
        dz = da.float()
        if a is not None:
            dz = dz * _mask_of(a, da.shape)
        elif relu_from_y:
            dz = dz * ((y.float() * st.scale + st.shift) > 0)
        dz2 = dz.reshape(-1, C)
        xh = (y.float().reshape(-1, C) - st.mean) * st.invstd
        s0, s1 = dz2.sum(0), (dz2 * xh).sum(0)
        dgamma.copy_(s1); dbeta.copy_(s0)
        dy = (gamma * st.invstd) * (dz2 - s0 / count - xh * (s1 / count))
        dy = dy.reshape(da.shape).to(torch.bfloat16)
        dy2 = None
        if y2 is not None:
            xh2 = (y2.float().reshape(-1, C) - st2.mean) * st2.invstd
            s2 = (dz2 * xh2).sum(0)
            dgamma2.copy_(s2); dbeta2.copy_(s0)
            dy2 = ((gamma2 * st2.invstd) * (dz2 - s0 / count - xh2 * (s2 / count))).reshape(da.shape).to(torch.bfloat16)
        dres = (da if premasked else dz.to(torch.bfloat16)) if want_dres else None
        return dy, dy2, dres
    M = da.numel() // C
    L = lib()
    msc = st.scale if (a is None and relu_from_y) else None
    msh = st.shift if (a is None and relu_from_y) else None
    if not reduced:
        L.bn_bwd_reduce(da, a, y, st.mean, st.invstd, y2, st2.mean if st2 else None, st2.invstd if st2 else None, M, C,
                        st.sums, st.shards, msc, msh)
    if _fused(st) and (a is None or a.dtype == torch.uint8):
        # finalize folded into the apply pass (sums zeroed by the state's BNPool at step start)
        dy = torch.empty_like(da)
        dy2 = torch.empty_like(da) if y2 is not None else None
        dres = torch.empty_like(da) if (want_dres and not premasked) else None
        g2 = [gamma2, st2.mean, st2.invstd, dgamma2, dbeta2] if y2 is not None else []
        L.bn_bwd_apply_fin(da, a, y, st.sums, st.shards, [gamma, st.mean, st.invstd, dgamma, dbeta], y2, g2, dy, dy2,
                           dres, M, C, msc, msh)
        if want_dres and premasked:
            dres = da
        return dy, dy2, dres
    L.bn_bwd_finalize(st.sums, st.shards, C, float(count), gamma, st.mean, st.invstd, gamma2,
                      st2.mean if st2 else None, st2.invstd if st2 else None, dgamma, dbeta, dgamma2, dbeta2, st.coef,
                      st2.coef if st2 else None)
    dy = torch.empty_like(da)
    dy2 = torch.empty_like(da) if y2 is not None else None
    dres = torch.empty_like(da) if (want_dres and not premasked) else None
    L.bn_bwd_apply(da, a, y, st.coef, dy, y2, st2.coef if st2 else None, dy2, dres, M, C, msc, msh)
    if want_dres and premasked:
        dres = da  # d(identity residual) = dz = da
    return dy, dy2, dres
