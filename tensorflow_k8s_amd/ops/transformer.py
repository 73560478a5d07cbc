"""Transformer ops (csrc/kernels/attention.hip, transformer.hip): LayerNorm, embeddings, fused
multi-head attention. bf16 activations, f32 statistics/gradients of parameters.

Attention operands are *column views* of 2-D token-major buffers: ``(buf, col)`` means the
[B*S, H*64] block of ``buf[:, col:col + H*64]`` -- e.g. q/k/v straight out of a fused QKV
projection ``qkv[B*S, 3*H*64]`` (q at col 0, k at H*64, v at 2*H*64). No head transposes.
CPU paths are fp32 references with the same rounding points and (for dropout) the same hash RNG.
"""
from __future__ import annotations

import math

import torch

from ._lib import lib, on_gpu
from .elementwise import eff_seed

HEAD_DIM = 64

# ----------------------------------------------------------------------------- LayerNorm


def layernorm_fwd(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-12,
                  mx_out: bool = False, skip_y: bool = False):
    """Returns (y bf16, mean f32 [M], rstd f32 [M]). mx_out (fp8 training): the kernel also writes
    MX(y) and MX(y^T), registered for the fp8 GEMMs that consume y (ops.fp8 _register_out);
    skip_y: ... and no bf16 y (every consumer is such a GEMM; ops.fp8 guards bf16 reads)."""
    W = x.shape[-1]
    x2 = x.reshape(-1, W)
    M = x2.shape[0]
    mx_out = mx_out and M % 32 == 0 and W % 32 == 0 and W <= 1024
    if not on_gpu(x):
        xf = x2.float()
        mu = xf.mean(1)
        var = ((xf - mu[:, None]) ** 2).mean(1)
        rs = torch.rsqrt(var + eps)
        y = ((xf - mu[:, None]) * rs[:, None] * gamma + beta).to(torch.bfloat16)
        y = y.reshape(x.shape)
        if mx_out:
            from . import fp8 as F8
            F8._register_out(y, *F8.mx_quantize_dual(y.reshape(M, W)))
        return y, mu, rs
    y = torch.empty_like(x)
    mean = torch.empty(M, dtype=torch.float32, device=x.device)
    rstd = torch.empty(M, dtype=torch.float32, device=x.device)
    if mx_out:
        from . import fp8 as F8
        qr, sr, qc, sc = F8._mx_bufs(M, W, x.device)
        lib().layernorm_fwd_mx(x2, gamma, beta, None if skip_y else y, mean, rstd, M, W, eps, qr, sr, qc, sc)
        F8._register_out(y, (qr, sr), (qc, sc))
        if skip_y:
            F8.mark_no_c(y)
        return y, mean, rstd
    lib().layernorm_fwd(x2, gamma, beta, y, mean, rstd, M, W, eps)
    return y, mean, rstd


def _zero_pair(a: torch.Tensor, b: torch.Tensor) -> None:
    """Zero two 1-D f32 gradient views with one fill when they are adjacent in the same storage, in
    either order (gamma/beta of one LayerNorm are consecutive in the flat arena; ParamArena places
    parameters in reverse registration order, so beta precedes gamma): saves a launch per LN."""
    if (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.device == b.device
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()):
        if b.storage_offset() == a.storage_offset() + a.numel():
            a.as_strided((a.numel() + b.numel(),), (1,), a.storage_offset()).zero_()
            return
        if a.storage_offset() == b.storage_offset() + b.numel():
            b.as_strided((a.numel() + b.numel(),), (1,), b.storage_offset()).zero_()
            return
    a.zero_(); b.zero_()


def layernorm_bwd(dy, x, gamma, mean, rstd, dgamma, dbeta, dres=None, accumulate: bool = False, drop=None,
                  dbias=None, mx_out: bool = False):
    """dx (+ dres) bf16; dgamma/dbeta (f32, written or accumulated). drop=(p, seed): also return
    dropout(dx, p, seed) (the consumer's dropout backward, written by the same kernel) -> (dx, dxd).
    dbias (f32 [W]): += column sums of the returned consumer gradient (dxd, else dx) -- the
    consuming Linear's bias gradient, reduced in the same kernel. mx_out (fp8 training): the kernel
    also writes MX row / column blocks of that consumer gradient (ops.fp8 _register_out), which the
    consumer's fp8 backward takes instead of quantizing it."""
    if drop is not None and drop[0] <= 0.0:
        dx = layernorm_bwd(dy, x, gamma, mean, rstd, dgamma, dbeta, dres, accumulate, dbias=dbias, mx_out=mx_out)
        return dx, dx
    W = x.shape[-1]
    M = x.numel() // W
    if not on_gpu(dy):
        d = dy.reshape(-1, W).float()
        xh = (x.reshape(-1, W).float() - mean[:, None]) * rstd[:, None]
        g = d * gamma
        dx = rstd[:, None] * (g - g.mean(1, keepdim=True) - xh * (g * xh).mean(1, keepdim=True))
        if dres is not None:
            dx = dx + dres.reshape(-1, W).float()
        dg, db = (d * xh).sum(0), d.sum(0)
        if accumulate:
            dgamma.add_(dg); dbeta.add_(db)
        else:
            dgamma.copy_(dg); dbeta.copy_(db)
        dx = dx.to(torch.bfloat16).reshape(dy.shape)
        mx_out = mx_out and M % 32 == 0 and W % 32 == 0 and W <= 1024
        if drop is not None:
            from .elementwise import dropout
            dxd = dropout(dx, drop[0], drop[1])
            if dbias is not None:
                dbias.add_(dxd.reshape(-1, W).float().sum(0))
            if mx_out:
                from . import fp8 as F8
                F8._register_out(dxd, *F8.mx_quantize_dual(dxd.reshape(M, W)))
            return dx, dxd
        if dbias is not None:
            dbias.add_(dx.reshape(-1, W).float().sum(0))
        if mx_out:
            from . import fp8 as F8
            F8._register_out(dx, *F8.mx_quantize_dual(dx.reshape(M, W)))
        return dx
    if not accumulate:
        _zero_pair(dgamma, dbeta)
    dx = torch.empty_like(dy)
    dxd = torch.empty_like(dy) if drop is not None else None
    mo = None
    if mx_out and M % 32 == 0 and W % 32 == 0 and W <= 1024:
        from . import fp8 as F8
        mo = F8._mx_bufs(M, W, dy.device)
    lib().layernorm_bwd(dy, x, gamma, mean, rstd, dres, dx, dgamma, dbeta, M, W, dxd,
                        float(drop[0]) if drop is not None else 0.0, int(drop[1]) if drop is not None else 0,
                        dbias=dbias, mx_out=list(mo) if mo else None)
    if mo:
        F8._register_out(dxd if drop is not None else dx, (mo[0], mo[1]), (mo[2], mo[3]))
    return (dx, dxd) if drop is not None else dx


# ----------------------------------------------------------------------------- embeddings


def embedding_fwd(ids, word, pos=None, seq_len: int = 1, type_ids=None, type_table=None, scale: float = 1.0):
    """out[t] = word[ids[t]]*scale (+ pos[t % seq_len]) (+ type_table[type_ids[t]]); bf16 [T, W]."""
    T = ids.numel()
    W = word.shape[1]
    if not on_gpu(word):
        o = word.float()[ids.reshape(-1).long().clamp(0, word.shape[0] - 1)] * scale
        if pos is not None:
            o = o + pos.float()[:seq_len].repeat(T // seq_len, 1)
        if type_table is not None:
            o = o + type_table.float()[type_ids.reshape(-1).long()]
        return o.to(torch.bfloat16)
    out = torch.empty(T, W, dtype=torch.bfloat16, device=word.device)
    lib().embedding_fwd(ids, word, pos, seq_len, type_ids, type_table, out, scale)
    return out


def embedding_bwd(ids, dy, dword, dpos=None, seq_len: int = 1, type_ids=None, dtype_table=None, scale: float = 1.0):
    """dword (+)= scatter of dy rows (f32 atomics: the caller zeroes or pre-writes dword);
    dpos[:seq_len] = column sums over the batch (overwritten); dtype_table (+)= per-type sums."""
    W = dy.shape[-1]
    if not on_gpu(dy):
        d = dy.reshape(-1, W).float()
        dword.view(-1, W).index_add_(0, ids.reshape(-1).long(), d * scale)
        if dpos is not None:
            dpos.view(-1, W)[:seq_len].copy_(d.view(-1, seq_len, W).sum(0))
        if dtype_table is not None:
            dtype_table.view(-1, W).index_add_(0, type_ids.reshape(-1).long(), d)
        return
    lib().embedding_bwd(ids, dy, dword, dpos, seq_len, type_ids, dtype_table, W, scale)


# ----------------------------------------------------------------------------- attention

def gather_rows(src: torch.Tensor, pos: torch.Tensor | None, S: int) -> torch.Tensor:
    """Prediction-head rows of a [B*S, W] activation: row (r // P) * S + pos[b, r % P] for pos int32
    [B, P] (BERT's MLM positions), or the first row of every sequence (pos None: the [CLS] rows)."""
    W = src.shape[-1]
    src2 = src.reshape(-1, W)
    B = src2.shape[0] // S
    P = pos.shape[-1] if pos is not None else 1
    if not on_gpu(src):
        rows = torch.arange(B, device=src.device)[:, None] * S
        rows = (rows + pos.long().reshape(B, P)) if pos is not None else rows
        return src2.index_select(0, rows.reshape(-1))
    out = torch.empty(B * P, W, dtype=src.dtype, device=src.device)
    lib().gather_rows(src2, pos.reshape(-1) if pos is not None else None, P, S, out)
    return out


def scatter_add_rows(dst: torch.Tensor, src: torch.Tensor, pos: torch.Tensor | None, S: int) -> None:
    """dst[(r // P) * S + pos[b, r % P]] += src[r] (the backward of gather_rows; repeated positions
    inside a sequence accumulate). dst [B*S, W] bf16, summed in f32 per add."""
    W = src.shape[-1]
    dst2 = dst.reshape(-1, W)
    P = pos.shape[-1] if pos is not None else 1
    B = src.shape[0] // P
    if not on_gpu(dst):
        rows = torch.arange(B, device=dst.device)[:, None] * S
        rows = (rows + pos.long().reshape(B, P)) if pos is not None else rows
        acc = dst2.float()
        acc.index_add_(0, rows.reshape(-1), src.reshape(-1, W).float())
        dst2.copy_(acc.to(dst.dtype))
        return
    lib().scatter_add_rows(dst2, src.reshape(-1, W), pos.reshape(-1) if pos is not None else None, P, S)


def _hash32(x: torch.Tensor) -> torch.Tensor:
    """Bit-exact torch (int64 holding uint32) copy of common.h hash32 (lowbias32)."""
    m = 0xFFFFFFFF
    x = x & m
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & m
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & m
    return x ^ (x >> 16)


def attn_drop_thr(p: float) -> int:
    """8-bit drop threshold of the attention-dropout mask (attention.hip drop_thr)."""
    return min(255, int(p * 256.0 + 0.5))


def attn_keep_scale(p: float) -> float:
    """Inverse keep probability of the quantized mask: 256 / (256 - thr) (exactly unbiased)."""
    return 256.0 / (256 - attn_drop_thr(p))


def dropout_keep_mask(seed: int, B: int, H: int, Sq: int, Sk: int, p: float) -> torch.Tensor:
    """The kernels' attention-dropout mask (bool [B,H,Sq,Sk]), bit-exact (attention.hip keep4_*):
    one hash32 per (group of 4 queries, key), folded with a per-head seed hash; byte q % 4 of it
    decides query q (kept iff byte >= round(256 p))."""
    s = int(seed) & 0xFFFFFFFFFFFFFFFF
    base = (s & 0xFFFFFFFF) ^ (s >> 32)
    bh = torch.arange(B * H, dtype=torch.int64)
    hs = _hash32(base ^ ((bh * 0x9E3779B9) & 0xFFFFFFFF))
    q = torch.arange(Sq, dtype=torch.int64)
    idx = ((q >> 2)[:, None] * Sk + torch.arange(Sk, dtype=torch.int64)[None, :]).reshape(-1)
    h = _hash32(hs[:, None] ^ idx[None, :]).reshape(B * H, Sq, Sk)
    byte = (h >> (8 * (q & 3))[None, :, None]) & 0xFF
    return (byte >= attn_drop_thr(p)).reshape(B, H, Sq, Sk)


def _view(buf, col, B, S, H):
    return buf.reshape(B * S, -1)[:, col:col + H * HEAD_DIM].reshape(B, S, H, HEAD_DIM)


def _ref_probs(q, k, kv_len, causal, scale):
    B, Sq, H, _ = q.shape
    Sk = k.shape[1]
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    mask = torch.zeros(B, 1, Sq, Sk, dtype=torch.bool)
    if kv_len is not None:
        mask |= torch.arange(Sk)[None, None, None, :] >= kv_len.long().cpu()[:, None, None, None]
    if causal:
        mask |= torch.arange(Sk)[None, :] > torch.arange(Sq)[:, None]
    s = s.masked_fill(mask, float("-inf"))
    return torch.softmax(s, -1).nan_to_num(0.0)


class AttnSpec:
    """Geometry of one attention call: q/k/v column views of token-major buffers."""

    def __init__(self, B, H, Sq, Sk, q, k, v, kv_len=None, causal=False, p_drop=0.0, seed=0, scale=None):
        self.B, self.H, self.Sq, self.Sk = B, H, Sq, Sk
        self.q, self.k, self.v = q, k, v  # (buf, col)
        self.kv_len, self.causal, self.p_drop, self.seed = kv_len, causal, p_drop, seed
        self.scale = scale if scale is not None else 1.0 / math.sqrt(HEAD_DIM)

    def strides(self):
        out = []
        for (buf, _), S in ((self.q, self.Sq), (self.k, self.Sk), (self.v, self.Sk)):
            rs = buf.shape[-1]
            out += [S * rs, rs]
        return out


def attention_fwd(sp: AttnSpec):
    """Returns (out bf16 [B*Sq, H*64], lse f32 [B,H,Sq])."""
    B, H, Sq, Sk = sp.B, sp.H, sp.Sq, sp.Sk
    dev = sp.q[0].device
    if not on_gpu(sp.q[0]):
        q, k, v = (_view(b, c, B, S, H).float() for (b, c), S in ((sp.q, Sq), (sp.k, Sk), (sp.v, Sk)))
        pr = _ref_probs(q, k, sp.kv_len, sp.causal, sp.scale)
        s = torch.einsum("bqhd,bkhd->bhqk", q, k) * sp.scale
        lse = torch.logsumexp(s.masked_fill(pr == 0, float("-inf")), -1)
        if sp.p_drop > 0:
            pr = pr * dropout_keep_mask(eff_seed(sp.seed), B, H, Sq, Sk, sp.p_drop) * attn_keep_scale(sp.p_drop)
        o = torch.einsum("bhqk,bkhd->bqhd", pr, v).reshape(B * Sq, H * HEAD_DIM)
        return o.to(torch.bfloat16), lse
    out = torch.empty(B * Sq, H * HEAD_DIM, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(B, H, Sq, dtype=torch.float32, device=dev)
    st = sp.strides() + [Sq * H * HEAD_DIM, H * HEAD_DIM]
    lib().attn_fwd(sp.q[0], sp.q[1], sp.k[0], sp.k[1], sp.v[0], sp.v[1], out, lse, [B, H, Sq, Sk], st, sp.kv_len,
                   sp.scale, sp.causal, sp.p_drop, sp.seed)
    return out, lse


def attention_bwd(sp: AttnSpec, out, dout, lse, dq, dk, dv):
    """dq/dk/dv: (buf, col) views to write (e.g. column slices of a fused dQKV buffer)."""
    B, H, Sq, Sk = sp.B, sp.H, sp.Sq, sp.Sk
    if not on_gpu(out):
        q, k, v = (_view(b, c, B, S, H).float().requires_grad_(True)
                   for (b, c), S in ((sp.q, Sq), (sp.k, Sk), (sp.v, Sk)))
        with torch.enable_grad():
            pr = _ref_probs(q, k, sp.kv_len, sp.causal, sp.scale)
            if sp.p_drop > 0:
                pr = pr * dropout_keep_mask(eff_seed(sp.seed), B, H, Sq, Sk, sp.p_drop) * attn_keep_scale(sp.p_drop)
            o = torch.einsum("bhqk,bkhd->bqhd", pr, v)
            gq, gk, gv = torch.autograd.grad(o, (q, k, v), dout.float().reshape(B, Sq, H, HEAD_DIM))
        for (buf, col), g, S in ((dq, gq, Sq), (dk, gk, Sk), (dv, gv, Sk)):
            _view(buf, col, B, S, H).copy_(g.to(torch.bfloat16))
        return
    delta = torch.empty(B, H, Sq, dtype=torch.float32, device=out.device)
    st = sp.strides() + [Sq * H * HEAD_DIM, H * HEAD_DIM]
    gst = []
    for (buf, _), S in ((dq, Sq), (dk, Sk), (dv, Sk)):
        rs = buf.shape[-1]
        gst += [S * rs, rs]
    lib().attn_bwd(sp.q[0], sp.q[1], sp.k[0], sp.k[1], sp.v[0], sp.v[1], out, dout, lse, delta, dq[0], dq[1], dk[0],
                   dk[1], dv[0], dv[1], [B, H, Sq, Sk], st, gst, sp.kv_len, sp.scale, sp.causal, sp.p_drop, sp.seed)
