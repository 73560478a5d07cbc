"""MX-fp8 linear layers (csrc/kernels/fp8.hip): OCP e4m3 values with one e8m0 (power-of-two)
scale per 32 K-elements of each row, multiplied by gfx950's block-scaled MFMA
(v_mfma_scale_f32_16x16x128_f8f6f4, 2x the bf16 MFMA rate).

Used for all three GEMMs of a linear layer of the transformer models when ``fp8=True``:

* forward   y  = X  W^T : X quantized along K (rows of X), W along K (rows of W);
* dgrad     dX = dY W   : dY quantized along N (its rows), W^T along N (``mx_quantize_t`` of W);
* wgrad     dW = dY^T X : dY^T and X^T quantized along the token dimension (``mx_quantize_t``).

MX blocks always run along the GEMM's reduction dimension, so the backward operands are produced
by a transposing quantizer (one LDS-staged pass, csrc/kernels/fp8.hip). The f32 master weights and
the optimizer stay f32; the weight gradient is accumulated in f32 by the GEMM epilogue. Shapes
that do not tile (reduction dim % 128, transposed rows % 32) fall back to the bf16 GEMMs. The CPU
path is the exact dequantized reference of the same quantization.
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


def mx_quantize_dual(x: torch.Tensor):
    """bf16 [R, C] (R, C % 32 == 0) -> (MX of x along C, MX of x^T along R) from ONE read of x:
    ((q [R, C], s [R, C/32]), (qt [C, R], st [C, R/32]))."""
    R, C = x.shape
    if R % MX_BLOCK or C % MX_BLOCK:
        raise ValueError(f"dual MX quantization needs R, C % 32 == 0, got {R}x{C}")
    if not on_gpu(x):
        return mx_quantize(x), mx_quantize(x.t().contiguous())
    q = torch.empty(R, C, dtype=torch.uint8, device=x.device)
    s = torch.empty(R, C // MX_BLOCK, dtype=torch.uint8, device=x.device)
    qt = torch.empty(C, R, dtype=torch.uint8, device=x.device)
    st = torch.empty(C, R // MX_BLOCK, dtype=torch.uint8, device=x.device)
    lib().mx_quant_dual(x.contiguous(), q, s, qt, st, R, C)
    return (q, s), (qt, st)


class GroupQuantizer:
    """Both MX quantizations of MANY bf16 tensors (a model's fp8 weights) in ONE launch per step
    (csrc/kernels/fp8.hip mx_quant_dual_kernel<true>: a device table of per-tensor descriptors,
    resident blocks walk all tensors' 128x128 tiles). Per-weight launches cost ~8 us each on the
    1024x1024..4096x1024 Transformer-big weights (67 of them per step) at a fraction of the HBM
    rate. Output buffers and the table are allocated once (fixed addresses: hipGraph-capturable).
    ``run()`` registers each weight's (MX(w), MX(w^T)) for this step's linear_fwd_mx (lookup by
    data pointer) and its backward (save_t)."""

    def __init__(self, weights: list[torch.Tensor]):
        self.ws = [w for w in weights]
        for w in self.ws:
            R, C = w.shape
            if R % MX_BLOCK or C % MX_BLOCK or not w.is_contiguous():
                raise ValueError(f"group MX quantization needs contiguous [R, C] with R, C % 32 == 0, got {tuple(w.shape)}")
        dev = self.ws[0].device
        self.out = []
        for w in self.ws:
            R, C = w.shape
            self.out.append(((torch.empty(R, C, dtype=torch.uint8, device=dev),
                              torch.empty(R, C // MX_BLOCK, dtype=torch.uint8, device=dev)),
                             (torch.empty(C, R, dtype=torch.uint8, device=dev),
                              torch.empty(C, R // MX_BLOCK, dtype=torch.uint8, device=dev))))
        self.table, self.total = None, 0
        if on_gpu(self.ws[0]):
            rows, t0 = [], 0
            for w, ((q, s), (qt, st)) in zip(self.ws, self.out):
                R, C = w.shape
                tc, tr = -(-C // 128), -(-R // 128)
                rows.append([w.data_ptr(), q.data_ptr(), s.data_ptr(), qt.data_ptr(), st.data_ptr(),
                             R | (C << 32), t0 | (tc << 32)])
                t0 += tc * tr
            self.total = t0
            self.table = torch.tensor(rows, dtype=torch.int64).to(dev)

    def run(self) -> None:
        if self.table is not None:
            lib().mx_quant_dual_group(self.table, len(self.ws), self.total)
        else:
            for w, ((q, s), (qt, st)) in zip(self.ws, self.out):
                (q_, s_), (qt_, st_) = mx_quantize_dual(w)
                q.copy_(q_); s.copy_(s_); qt.copy_(qt_); st.copy_(st_)
        for w, o in zip(self.ws, self.out):
            _WQ[w.data_ptr()] = (w, tuple(w.shape), o)


# this step's pre-quantized weights (GroupQuantizer.run): data pointer -> (w, shape, (MX(w), MX(w^T)))
_WQ: dict[int, tuple] = {}


def _shape2(x: torch.Tensor) -> tuple:
    """The [rows, last] view every fp8 GEMM takes of an operand (keys of the per-step caches)."""
    return (x.numel() // x.shape[-1], x.shape[-1]) if x.dim() else (1, 1)


# Transposed MX operands produced in the forward for the backward of the same step: the forward
# quantizes its input x and weight w in both directions with one read each (mx_quantize_dual) and
# parks MX(x^T) (weight-gradient operand) and MX(w^T) (dgrad operand) here, keyed by the data
# pointer of the tensor the backward will pass. An entry holds a reference to its source tensor,
# so that memory cannot be reused by another tensor while the entry exists; the backward pops it.
_SAVED: dict[int, tuple] = {}


def save_t(x: torch.Tensor, qt) -> None:
    """Park MX(x^T) for this step's backward. The same tensor may feed several fp8 GEMMs (the
    encoder memory feeds every decoder layer's cross-attention K/V): the entry is counted and
    outlives the backward's take_t of every use."""
    if len(_SAVED) > 4096:  # forwards without backwards (evaluation): do not grow without bound
        _SAVED.clear()
    k = x.data_ptr()
    e = _SAVED.get(k)
    if e is not None and e[1] == _shape2(x) and e[2] is qt:
        e[3] += 1
    else:
        _SAVED[k] = [x, _shape2(x), qt, 1]


def take_t(x: torch.Tensor):
    e = _SAVED.get(x.data_ptr())
    if e is None or e[1] != _shape2(x):
        return None
    e[3] -= 1
    if e[3] <= 0:
        del _SAVED[x.data_ptr()]
    return e[2]


# this step's MX quantizations of fp8 GEMM inputs, keyed by (data pointer, shape); an entry holds
# its source tensor, so the memory cannot be reused by another tensor while it exists
_XQ: dict[tuple, tuple] = {}


def clear_saved() -> None:
    _SAVED.clear()
    _WQ.clear()
    _XQ.clear()
    _NO_C.clear()


def linear_fwd_mx(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
                  resid: torch.Tensor | None = None, aux: torch.Tensor | None = None, drop_p: float = 0.0,
                  drop_seed: int = 0, wq=None, save: bool = False, mx_out: bool = False,
                  mx_skip_c: bool = False) -> torch.Tensor:
    """y[M,N] = dropout(act(MX(x) @ MX(w)^T + bias)) (+ resid), bf16 out. wq: pre-quantized weight.
    save: also produce MX(x^T) / MX(w^T) for this step's backward (save_t) where it will use fp8.
    mx_out: the epilogue also writes MX(y) and MX(y^T) (registered for the next fp8 GEMM on y, see
    _register_out); mx_skip_c: ... and no bf16 y (the caller guarantees every consumer is such a GEMM)."""
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M, N = x2.shape[0], w.shape[0]
    if K % 128:
        raise ValueError(f"MX-fp8 GEMM needs K % 128 == 0, got {K}")
    dg_ok, wg_ok = mx_backward_ok(M, N, K)
    if wq is None and save:
        # this step's pre-quantized weights are valid only inside the training step that quantized
        # them (an evaluation forward after the optimizer update must not see last step's MX(w))
        e = _WQ.get(w.data_ptr())
        if e is not None and e[1] == tuple(w.shape):
            wq = e[2][0]
            if save and dg_ok:
                save_t(w, e[2][1])
    # training forwards only: an input saved for this step's backward is immutable until then, so a
    # second GEMM on the same tensor (the decoders' encoder memory) reuses its quantization
    key = (x2.data_ptr(), _shape2(x2))
    xe = _XQ.get(key) if save and wg_ok else None
    if xe is not None:
        (xq, xs), xt = xe[1], xe[2]
        save_t(x2, xt)
    elif save and wg_ok:
        _check_stored(x2)
        (xq, xs), xt = mx_quantize_dual(x2)
        save_t(x2, xt)
        _XQ[key] = (x2, (xq, xs), xt)
    else:
        _check_stored(x2)
        xq, xs = mx_quantize(x2)
    if wq is not None:
        wq_, ws_ = wq
    elif save and dg_ok and w.is_contiguous():
        (wq_, ws_), wt = mx_quantize_dual(w)
        save_t(w, wt)
    else:
        wq_, ws_ = mx_quantize(w)
    mx_out = mx_out and M % MX_BLOCK == 0 and N % MX_BLOCK == 0
    if not on_gpu(x):
        y = mx_dequantize(xq, xs) @ mx_dequantize(wq_, ws_).t()
        if bias is not None:
            y = y + bias.float()
        if aux is not None:
            from .gemm import store_aux_ref
            store_aux_ref(aux, y, N)
        y = act_ref(y, act)
        if drop_p > 0:
            from .elementwise import dropout_keep, eff_seed, keep_scale
            y = y * dropout_keep(eff_seed(drop_seed), y.numel(), drop_p).reshape(y.shape) * keep_scale(drop_p)
        y = y.to(torch.bfloat16)
        if resid is not None:
            y = (y.float() + resid.reshape(-1, N).float()).to(torch.bfloat16)
        if mx_out:
            _register_out(y, *mx_quantize_dual(y))
            if mx_skip_c:
                _poison_no_c(y)
        return y
    y = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    mo = _mx_bufs(M, N, y.device) if mx_out else None
    lib().gemm_mxfp8(xq, xs, wq_, ws_, y, M, N, K, bias, resid.reshape(-1, N) if resid is not None else None,
                     ACT[act], aux, drop_p, drop_seed, mx_out=list(mo) if mo else None, mx_skip_c=bool(mo and mx_skip_c))
    if mo:
        _register_out(y, (mo[0], mo[1]), (mo[2], mo[3]))
        if mx_skip_c:
            mark_no_c(y)
    return y


def _mx_bufs(M: int, N: int, dev):
    """Epilogue MX outputs of a bf16 [M, N]: (qr [M, N], sr [M, N/32], qc [N, M], sc [N, M/32])."""
    return (torch.empty(M, N, dtype=torch.uint8, device=dev), torch.empty(M, N // MX_BLOCK, dtype=torch.uint8, device=dev),
            torch.empty(N, M, dtype=torch.uint8, device=dev), torch.empty(N, M // MX_BLOCK, dtype=torch.uint8, device=dev))


def _register_out(y: torch.Tensor, rowq, colq) -> None:
    """A GEMM output whose MX copies its producer already wrote: the next linear_fwd_mx on y (training)
    and fp8 backward operands of y (cached_dual) take them instead of quantizing y again."""
    _XQ[(y.data_ptr(), _shape2(y))] = (y, rowq, colq)


# outputs whose bf16 values were never stored (mx_skip_c): only their MX copies may be used
_NO_C: set = set()


def mark_no_c(y: torch.Tensor) -> None:
    """y's bf16 values were never stored (only its MX copies, _register_out)."""
    _NO_C.add((y.data_ptr(), _shape2(y)))


def _check_stored(x: torch.Tensor) -> None:
    if _NO_C and (x.data_ptr(), _shape2(x)) in _NO_C:
        raise RuntimeError("fp8: a GEMM output produced with mx_skip_c (no bf16 values) reached a consumer "
                           "that reads bf16 -- produce it with mx_skip_c=False")


def check_stored(*xs: torch.Tensor) -> None:
    """Raise if any of xs is an MX-only output (its bf16 values were never stored)."""
    for x in xs:
        if x is not None:
            _check_stored(x.reshape(-1, x.shape[-1]))


def _poison_no_c(y: torch.Tensor) -> None:
    """CPU emulation of mx_skip_c: the GPU epilogue never stores y's bf16 values, so the reference
    path makes them NaN and marks y -- a bf16 consumer then raises (_check_stored) or, if it bypasses
    the check, poisons the loss, exactly as the unwritten device memory would."""
    y.fill_(float("nan"))
    mark_no_c(y)


def cached_dual(y: torch.Tensor):
    """(MX(y), MX(y^T)) of y when its producer emitted them this step, else None."""
    e = _XQ.get((y.data_ptr(), _shape2(y)))
    return (e[1], e[2]) if e is not None and e[2] is not None else None


def mx_quantize_t(x: torch.Tensor):
    """bf16 [R, C] (R % 32 == 0) -> MX of x^T: (q uint8 [C, R], s uint8 [C, R/32])."""
    R, C = x.shape
    if R % MX_BLOCK:
        raise ValueError(f"transposed MX quantization needs rows % 32 == 0, got {R}")
    if not on_gpu(x):
        return mx_quantize(x.t().contiguous())
    q = torch.empty(C, R, dtype=torch.uint8, device=x.device)
    s = torch.empty(C, R // MX_BLOCK, dtype=torch.uint8, device=x.device)
    lib().mx_quant_t(x.contiguous(), q, s, R, C)
    return q, s


# Weight gradients in MX-fp8 (True) or bf16 (False) in the fp8 models. A/B switch for tools and
# bench.py --mx-wgrad; the default is the faster in-model measurement (profiles/perf_log_r5.md).
MX_WGRAD = True


def mx_backward_ok(M: int, N: int, K: int) -> tuple[bool, bool]:
    """(dgrad, wgrad) eligibility of a [M tokens, K in] x [N out, K in] linear layer: the
    reduction dims (N for dgrad, M for wgrad) must be multiples of 128 (one scaled-MFMA K-tile)."""
    return N % 128 == 0 and K % 8 == 0, MX_WGRAD and M % 128 == 0


def linear_dgrad_mx(dy: torch.Tensor, w: torch.Tensor, resid: torch.Tensor | None = None,
                    dact_src: torch.Tensor | None = None, dact: str | None = None, wt=None, dyq=None,
                    drop_p: float = 0.0, drop_seed: int = 0, mx_out: bool = False,
                    colsum: torch.Tensor | None = None, mx_skip_c: bool = False) -> torch.Tensor:
    """dx[M,K] = dropout((MX(dy) @ MX(w^T)^T) [* act'(dact_src)]) (+ resid), bf16 -- the bf16
    linear_dgrad's epilogue order. wt: pre-quantized w^T (else the one the forward saved, else
    quantized here); dyq: pre-quantized dy. colsum: as ops.gemm.linear_dgrad. mx_skip_c (with
    mx_out): no bf16 dx -- every consumer takes the MX copies."""
    M, N = dy.shape
    K = w.shape[1]
    if dyq is None:
        _check_stored(dy)
    dq, ds = dyq if dyq is not None else mx_quantize(dy)
    if wt is None:
        wt = take_t(w)
    wq_, ws_ = wt if wt is not None else mx_quantize_t(w)
    if not on_gpu(dy):
        from .gemm import act_grad_ref
        y = mx_dequantize(dq, ds) @ mx_dequantize(wq_, ws_).t()
        if dact_src is not None:
            y = y * act_grad_ref(dact_src if dact_src.dtype == torch.uint8 else dact_src.float(), dact)
        if drop_p > 0:
            from .elementwise import dropout_keep, eff_seed, keep_scale
            y = y * dropout_keep(eff_seed(drop_seed), y.numel(), drop_p).reshape(y.shape) * keep_scale(drop_p)
        y = y.to(torch.bfloat16)
        if colsum is not None:
            colsum.add_(y.float().sum(0))
        if resid is not None:
            y = (y.float() + resid.float()).to(torch.bfloat16)
        if mx_out and M % MX_BLOCK == 0 and K % MX_BLOCK == 0:
            _register_out(y, *mx_quantize_dual(y))
            fuse_cs = colsum is not None and resid is None and (dact_src is not None or drop_p > 0)
            if mx_skip_c and (colsum is None or fuse_cs):
                _poison_no_c(y)
        return y
    dx = torch.empty(M, K, dtype=torch.bfloat16, device=dy.device)
    mo = _mx_bufs(M, K, dx.device) if mx_out and M % MX_BLOCK == 0 and K % MX_BLOCK == 0 else None
    fuse_cs = colsum is not None and resid is None and (dact_src is not None or drop_p > 0)
    skip = bool(mo and mx_skip_c and (colsum is None or fuse_cs))
    lib().gemm_mxfp8(dq, ds, wq_, ws_, dx, M, K, N, None, resid, 0, None, drop_p, drop_seed,
                     dact_src=dact_src, dact=ACT[dact] if dact_src is not None else 0, mx_out=list(mo) if mo else None,
                     mx_skip_c=skip, colsum=colsum if fuse_cs else None)
    if mo:
        _register_out(dx, (mo[0], mo[1]), (mo[2], mo[3]))
        if skip:
            mark_no_c(dx)
    if colsum is not None and not fuse_cs:
        colsum.add_(dx.float().sum(0))
    return dx


def linear_wgrad_mx(dy: torch.Tensor, x: torch.Tensor, gw: torch.Tensor, accumulate: bool = False,
                    dyt=None) -> None:
    """gw[N,K] (f32) (+)= MX(dy^T) @ MX(x^T)^T (reduction over the M tokens). dyt: pre-quantized
    dy^T; x^T: the forward's saved one when present."""
    M, N = dy.shape
    K = x.shape[1]
    aq, as_ = dyt if dyt is not None else mx_quantize_t(dy)
    xt = take_t(x)
    if xt is None:
        _check_stored(x)
    bq, bs = xt if xt is not None else mx_quantize_t(x)
    if not on_gpu(dy):
        g = mx_dequantize(aq, as_) @ mx_dequantize(bq, bs).t()
        v = gw.view(N, K)
        v.add_(g) if accumulate else v.copy_(g)
        return
    splits = wgrad_splits(N, K, M)
    if splits == 1:
        lib().gemm_mxfp8(aq, as_, bq, bs, gw.view(N, K), N, K, M, None, None, 0, None, 0.0, 0,
                         beta=1.0 if accumulate else 0.0)
        return
    # split-K into f32 slabs, then one reduce pass (f32 atomics from the epilogue measured 2.5x
    # slower end to end: Transformer-big fp8 33.3 ms/step, 11 ms of it in atomic weight gradients)
    from . import _lib as _lib_mod
    stride = ((N * K + 3) // 4) * 4
    ws = _lib_mod.workspace(dy.device, splits * stride, slot=_lib_mod.WGRAD_SLOT)
    lib().gemm_mxfp8(aq, as_, bq, bs, ws, N, K, M, None, None, 0, None, 0.0, 0, splits=splits, split_stride=stride)
    lib().splitk_reduce(ws, splits, stride, N * K, gw.view(-1), None, accumulate, 1.0)


# split-K fill target (256x256 blocks; 2x for 128x128) and minimum K-tiles per split. (Unsplit
# 128x128 weight gradients were measured slower on Transformer-big -- 19.0 vs 18.86 ms,
# profiles/perf_log_r3c.md -- and removed.)
WGRAD_TARGET = 256
WGRAD_MIN_KT = 8


def wgrad_splits(N: int, K: int, M: int) -> int:
    """Split-K slabs of an fp8 weight gradient [N, K] reduced over M tokens: fill ~one round of
    256x256 blocks (two of 128x128 when a side is < 256) with >= 8 K-tiles of 128 per split; the
    count the g4 launcher will actually run (ceil(K-tiles / per-split))."""
    nkt = M // 128
    big = N >= 256 and K >= 256
    t = (-(-N // 256)) * (-(-K // 256)) if big else (-(-N // 128)) * (-(-K // 128))
    target = WGRAD_TARGET if big else 2 * WGRAD_TARGET
    s = max(1, min(-(-target // t), max(1, nkt // WGRAD_MIN_KT)))
    per = -(-nkt // s)
    return -(-nkt // per)
