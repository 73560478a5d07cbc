"""Matrix-multiply and NHWC convolution ops on the tfk MFMA implicit-GEMM engine (csrc/kernels/gemm.hip).

Layouts (MI355X-first, not a translation of TF's): activations NHWC bf16, conv weights OHWI bf16
([Cout][R][S][Cin], the K-contiguous "B" operand of the forward GEMM), linear weights [out][in].
All weight gradients are produced in f32 directly into the caller's (flat-arena) grad view.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from . import tuning
from . import _lib as _lib_mod
from ._lib import lib, on_gpu, workspace

A_KIN, A_KOUT, A_CONV_FWD, A_CONV_DGRAD = 0, 1, 2, 3
B_KIN, B_KOUT, B_CONV_WGRAD = 0, 1, 2
EPI_BF16, EPI_F32 = 0, 1
ACT = {None: 0, "none": 0, "relu": 1, "gelu": 2, "tanh": 3}


def act_ref(y: torch.Tensor, act) -> torch.Tensor:
    """f32 reference of the epilogue activations."""
    a = ACT[act]
    if a == 1:
        return torch.relu(y)
    if a == 2:
        return F.gelu(y, approximate="tanh")
    if a == 3:
        return torch.tanh(y)
    return y
NO_CONV = [0] * 15
TARGET_BLOCKS = int(os.environ.get("TFK_TARGET_BLOCKS", 1024))  # split-K fill target: ~4 blocks per CU on 256 CUs
SPLIT_MIN_KTILES = int(os.environ.get("TFK_SPLIT_MIN_KTILES", 4))  # min 64-deep K tiles per split
# Conv weight gradients issued on a side stream (runtime/streams.py) run concurrently with the
# input-gradient chain: their split-K fill target and tuned split counts (swept in isolation) are
# divided by SIDE_WGRAD_FILL_DIV so they hold fewer CU slots while the critical path's kernels wait
# for them. ResNet-50 bs256 step, same box, alternating: 1 -> 21.94 / 22.01 / 21.92 / 22.09 / 22.00,
# 2 -> 21.68 / 21.74 / 21.77 / 21.73 / 21.78, 3 -> 21.94 / 22.04 / 22.08, 4 -> 22.27 / 22.09 ms.
# Linear weight gradients likewise (Transformer-big 18.38 -> 18.18 ms/step, alternating).
SIDE_WGRAD_FILL_DIV = int(os.environ.get("TFK_SIDE_WGRAD_DIV", 2))
# Split-K for f32 outputs (weight gradients): per-split workspace slabs + splitk_reduce (two
# passes, bitwise deterministic). (f32 atomics from the epilogue were measured slower on MI355X,
# ResNet-50 bs256 step 39.4 vs 32.1 ms: hundreds of splits hammering one small gradient from all
# 8 XCDs serialise on the atomics.)


@dataclass(frozen=True)
class ConvGeom:
    N: int
    H: int
    W: int
    C: int
    K: int  # output channels
    R: int
    S: int
    sh: int = 1
    sw: int = 1
    ph: int = 0
    pw: int = 0
    dh: int = 1
    dw: int = 1

    @property
    def P(self) -> int:
        return (self.H + 2 * self.ph - self.dh * (self.R - 1) - 1) // self.sh + 1

    @property
    def Q(self) -> int:
        return (self.W + 2 * self.pw - self.dw * (self.S - 1) - 1) // self.sw + 1

    def vec(self):
        return [self.N, self.H, self.W, self.C, self.P, self.Q, self.K, self.R, self.S, self.sh, self.sw, self.ph,
                self.pw, self.dh, self.dw]

    @property
    def pointwise(self) -> bool:
        return self.R == 1 and self.S == 1 and self.sh == 1 and self.sw == 1 and self.ph == 0 and self.pw == 0

    def flops(self) -> int:
        return 2 * self.N * self.P * self.Q * self.K * self.R * self.S * self.C


# (bm, bn): (concurrent blocks on the chip, relative MFMA efficiency) of the register-staged engine
# (gemm.hip), measured by tools/gemm_bench.py in round 1.
_TILES = {(256, 256): (256, 0.76), (128, 128): (512, 0.62), (256, 64): (512, 0.60), (128, 64): (768, 0.45),
          (64, 64): (1024, 0.30), (64, 256): (512, 0.55)}
# The LDS-DMA engine (gemm_g4.hip) on the same scale, for the modes it serves (dense operands and the
# Cin % 64 == 0 conv-forward gather): tools/engine_bench.py on MI355X -- 256x256 (16 waves) ~1.0-1.3
# PF/s, 128x128 (4 waves, 2 blocks/CU) ~0.7-1.1 PF/s vs the register engine's 0.6-0.9.
_G4_TILES = {(256, 256): (256, 0.95), (128, 128): (512, 0.80), (128, 64): (768, 0.62), (64, 128): (768, 0.62)}
# 4-wave 64x256 / 256x64 blocks of the g4 engine for dense weight gradients with a narrow side
# (rect_ok): the register engine's 64x64 tile ran these at ~300 TF/s (ResNet-50 1x1 wgrads)
_G4_RECT = {(64, 256): (512, 0.80), (256, 64): (512, 0.80)}
G4_RECT = True
G4_BIG_MIN_K = 512  # one 16-wave block per CU: shorter K cannot amortise its prologue/epilogue
# 64x256 tile for Cout<=64 conv weight gradients whose B gather changes (r,s) every chunk (C <= 16,
# i.e. the 7x7 stem on C padded to 8). Measured on MI355X (ResNet-50 bs256, rocprofv3): stem wgrad
# 673 -> 644 us; the stage-1 3x3 (C=64) got slower on it (236 -> 249 us), so it keeps 64x64.
WIDE_WGRAD = True
WIDE_WGRAD_MAX_C = 16
BIG_TILE_MIN_K = 2048  # register engine: one 8-wave block per CU, needs a long K loop
G4_ENABLED = os.environ.get("TFK_GEMM_ENGINE", "g4") != "reg"


def pick_tile(M: int, N: int, splits_ok: bool = False, big_ok: bool = False, K: int = 0, mid_ok: bool = True,
              wide_ok: bool = False, split_target: int | None = None, g4: bool = False, narrow_ok: bool = False,
              rect_ok: bool = False):
    """Tile with the lowest modelled time: rounds of concurrent blocks x per-block work / efficiency
    (a 256x256 tile runs one block per CU; smaller tiles 2-4 blocks/CU at lower efficiency).
    big_ok: operand modes that have the 256x256 instantiation (dense, non-gather); K: reduction
    length. mid_ok: the mode has the 256x64 tile (every mode except the conv fwd/dgrad gathers).
    wide_ok: the mode has the 64x256 tile (conv weight gradient gather), only worth it for M <= 64.
    g4: the mode runs on the LDS-DMA engine (its 128x128 / 256x256 tiles; 256x256 also with split-K).
    narrow_ok: also its 2-wave 128x64 / 64x128 tiles (measured faster than the register engine
    for the im2col weight-gradient gather only; dense and BN-epilogue shapes keep the latter)."""
    g4 = g4 and G4_ENABLED
    best, best_cost = None, None
    cands = dict(_TILES)
    if g4:
        cands.update({t: v for t, v in _G4_TILES.items() if narrow_ok or t[0] == t[1]})
    rect = g4 and rect_ok and G4_RECT
    if rect:
        cands.update(_G4_RECT)
    for (bm, bn), (slots, eff) in cands.items():
        if rect and (bm, bn) in _G4_RECT:
            slots, eff = _G4_RECT[(bm, bn)]
        elif g4 and (bm, bn) in _G4_TILES and (narrow_ok or bm == bn):
            slots, eff = _G4_TILES[(bm, bn)]
            if (bm, bn) == (256, 256) and (M < 256 or N < 256 or K < G4_BIG_MIN_K):
                continue
        elif (bm, bn) == (256, 256) and (not big_ok or splits_ok or M < 256 or N < 256 or K < BIG_TILE_MIN_K):
            continue
        if (bm, bn) == (256, 64) and (not mid_ok or M < 256):
            continue
        if (bm, bn) == (64, 256) and not (rect and N >= 256) and (not wide_ok or M > 64 or N <= 128):
            continue
        if bn > 64 and N <= 64:
            continue
        tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
        s = pick_splits(tiles, K, target=split_target) if (splits_ok and K) else 1
        rounds = -(-tiles * s // slots)
        # seconds: MFMA work per round at eff x (2.3 PF / 256 CUs), a fixed prologue/epilogue
        # latency per round, and the f32 split-K slabs (written, then read by splitk_reduce)
        kb = max(K, 64) / s
        cost = rounds * ((slots / 256) * 2.0 * bm * bn * kb / (eff * 9.0e12) + 1.5e-6)
        if s > 1:
            cost += 2.0 * s * M * N * 4 / 4.0e12
        if best_cost is None or cost < best_cost * 0.98:
            best, best_cost = (bm, bn), cost
    return best


def pick_splits(tiles: int, K: int, min_ktiles: int | None = None, target: int | None = None) -> int:
    """Split-K count filling ~`target` blocks (default TARGET_BLOCKS) with >= min_ktiles K-tiles each."""
    min_ktiles = SPLIT_MIN_KTILES if min_ktiles is None else min_ktiles
    TARGET_BLOCKS = target or globals()["TARGET_BLOCKS"]
    nkt = (K + 63) // 64
    if tiles >= TARGET_BLOCKS // 2:
        return 1
    s = max(1, TARGET_BLOCKS // max(tiles, 1))
    s = min(s, max(1, nkt // min_ktiles))
    return s


def _gemm(A, B, C, M, N, K, lda, ldb, ldc, amode, bmode, epi, tile, *, alpha=1.0, beta=0.0, bias=None, resid=None,
          act=0, stats=None, shards=1, splits=1, batch=1, sA=0, sB=0, sC=0, split_stride=0, conv=NO_CONV, bnr=None,
          aux=None, dact_src=None, dact=0, drop_p=0.0, drop_seed=0, rowmap=(), colsum=None):
    lib().gemm(A, B, C, M, N, K, lda, ldb, ldc, amode, bmode, epi, tile[0], tile[1], alpha, beta, bias, resid, act,
               stats, shards, splits, batch, sA, sB, sC, split_stride, conv,
               bnr.gemm_args() if bnr is not None else [],
               (int(bnr.relu) | (2 if bnr.premask else 0)) if bnr is not None else 0,
               bnr.st.shards if bnr is not None else 1, aux, dact_src, dact, drop_p, drop_seed, list(rowmap), colsum)


def _f32_out_splitk(run, M: int, N: int, K: int, tiles: int, out: torch.Tensor, accumulate: bool, device,
                    force_splits: int | None = None, split_target: int | None = None, slot: str = "splitk"):
    """Run an f32-epilogue GEMM with split-K into a workspace, then reduce into `out` ([M][N] f32)."""
    splits = force_splits if force_splits is not None else pick_splits(tiles, K, target=split_target)
    ns = int(lib().gemm_splits(K, splits))
    if ns == 1:
        run(out, 1, 0, 1.0 if accumulate else 0.0)
        return
    stride = ((M * N + 3) // 4) * 4
    ws = workspace(device, ns * stride, slot=slot)
    run(ws, splits, stride, 0.0)
    lib().splitk_reduce(ws, ns, stride, M * N, out, None, accumulate, 1.0)


# =========================================================================== linear
def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, act: str | None = None,
               resid: torch.Tensor | None = None, out: torch.Tensor | None = None,
               aux: torch.Tensor | None = None, drop_p: float = 0.0, drop_seed: int = 0) -> torch.Tensor:
    """y[M,N] = dropout(act(x[M,K] @ w[N,K]^T + bias)) (+ resid). bf16 in/out, f32 accumulate.
    aux: also store the pre-activation (bf16) there, for the activation backward. Dropout mask =
    ops.elementwise.dropout_keep(eff_seed(drop_seed), M*N, drop_p) (backward: elementwise.dropout(dy));
    eff_seed adds the per-step device key of the running step (elementwise.rng_key)."""
    M, K = x.shape[0], x.shape[-1]
    N = w.shape[0]
    if not on_gpu(x):
        y = x.float().reshape(-1, K) @ w.float().t()
        if bias is not None:
            y = y + bias.float()
        if aux is not None:
            store_aux_ref(aux, y, N)
        y = act_ref(y, act)
        if drop_p > 0:
            from .elementwise import dropout_keep, eff_seed, keep_scale
            y = y * dropout_keep(eff_seed(drop_seed), y.numel(), drop_p).reshape(y.shape) * keep_scale(drop_p)
        y = y.to(torch.bfloat16)
        if resid is not None:
            y = (y.float() + resid.float()).to(torch.bfloat16)
        if out is not None:
            out.copy_(y)
            return out
        return y
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
    _gemm(x2, w, y, M, N, K, K, K, N, A_KIN, B_KIN, EPI_BF16, pick_tile(M, N, big_ok=True, K=K, g4=True), bias=bias, act=ACT[act],
          resid=resid.reshape(-1, N) if resid is not None else None, aux=aux, drop_p=drop_p, drop_seed=drop_seed)
    return y


def relu_mask_pack(z: torch.Tensor) -> torch.Tensor:
    """uint8 [rows, N/8] relu mask of pre-activations z [rows, N]: bit e of byte j = z[:, 8j+e] > 0
    (the GEMM epilogue's aux_bits layout; CPU reference)."""
    bits = (z.to(torch.bfloat16).float() > 0).reshape(z.shape[0], -1, 8).to(torch.int32)
    return (bits << torch.arange(8, dtype=torch.int32)).sum(-1).to(torch.uint8)


def relu_mask_unpack(m: torch.Tensor) -> torch.Tensor:
    """f32 [rows, 8 * cols] 0/1 relu' from a uint8 relu mask [rows, cols] (CPU reference)."""
    bits = (m.to(torch.int32).unsqueeze(-1) >> torch.arange(8, dtype=torch.int32)) & 1
    return bits.reshape(m.shape[0], -1).float()


def store_aux_ref(aux: torch.Tensor, y: torch.Tensor, N: int) -> None:
    """CPU reference of the epilogue's aux store: the bf16 pre-activation, or its relu mask (uint8 aux)."""
    if aux.dtype == torch.uint8:
        aux.view(-1, N // 8).copy_(relu_mask_pack(y.reshape(-1, N)))
    else:
        aux.view(-1, N).copy_(y)


def act_grad_ref(z: torch.Tensor, act: str | None) -> torch.Tensor:
    """f32 derivative of the activation at pre-activation z (CPU reference); z may be the uint8 relu
    mask (aux_bits) of a relu layer."""
    if z.dtype == torch.uint8:
        return relu_mask_unpack(z)
    z = z.float()
    if ACT[act] == 1:
        return (z > 0).float()
    if ACT[act] == 2:
        k0, k1 = 0.7978845608028654, 0.044715
        t = torch.tanh(k0 * (z + k1 * z ** 3))
        return 0.5 * (1 + t) + 0.5 * z * (1 - t * t) * k0 * (1 + 3 * k1 * z * z)
    if ACT[act] == 3:
        return 1 - torch.tanh(z) ** 2
    return torch.ones_like(z)


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, resid: torch.Tensor | None = None,
                 dact_src: torch.Tensor | None = None, dact: str | None = None, drop_p: float = 0.0,
                 drop_seed: int = 0, colsum: torch.Tensor | None = None) -> torch.Tensor:
    """dx[M,K] = dropout((dy[M,N] @ w[N,K]) * act'(dact_src)) (+ resid). drop_p/drop_seed: the
    backward of a forward dropout on this layer's INPUT (mask = ops.elementwise.dropout_keep(eff_seed(drop_seed),
    M*K, drop_p), e.g. the FFN's relu dropout) fused into the epilogue instead of a separate pass.
    colsum (f32 [K], with dact_src or dropout): += the column sums of dx before the residual add --
    the bias gradient of the layer that consumes dx, from the epilogue instead of a column pass."""
    N, K = w.shape
    dy2 = dy.reshape(-1, N)
    M = dy2.shape[0]
    if not on_gpu(dy):
        dx = dy2.float() @ w.float()
        if dact_src is not None:
            dx = dx * act_grad_ref(dact_src.reshape(dx.shape[0], -1), dact)
        if drop_p > 0:
            from .elementwise import dropout_keep, eff_seed, keep_scale
            dx = dx * dropout_keep(eff_seed(drop_seed), dx.numel(), drop_p).reshape(dx.shape) * keep_scale(drop_p)
        dx = dx.to(torch.bfloat16)
        if colsum is not None:
            colsum.add_(dx.float().sum(0))
        if resid is not None:
            dx = (dx.float() + resid.reshape(-1, K).float()).to(torch.bfloat16)
        return dx
    dx = torch.empty(M, K, dtype=torch.bfloat16, device=dy.device)
    fuse_cs = colsum is not None and resid is None and (dact_src is not None or drop_p > 0)
    plain = resid is None and dact_src is None and drop_p == 0.0
    if plain and _dgrad_splitk(dy2, w, dx, M, K, N):
        if colsum is not None:
            colsum.add_(dx.float().sum(0))
        return dx
    _gemm(dy2, w, dx, M, K, N, N, K, K, A_KIN, B_KOUT, EPI_BF16, pick_tile(M, K, big_ok=True, K=N, g4=K % 8 == 0),
          resid=resid.reshape(-1, K) if resid is not None else None,
          dact_src=dact_src.reshape(-1, K) if dact_src is not None else None,
          dact=ACT[dact] if dact_src is not None else 0, drop_p=drop_p, drop_seed=drop_seed,
          colsum=colsum if fuse_cs else None)
    if colsum is not None and not fuse_cs:
        colsum.add_(dx.float().sum(0))  # plain epilogue: no fused column sums
    return dx


# Plain input gradients whose output is too small to fill the chip with 256x256 tiles but whose
# reduction is long (the tied-logits dgrad: dx[8192][1024] over the 33728-wide vocabulary = 128
# tiles): split the reduction over the blocks, f32 slabs, one reduce pass writing the bf16 dx.
# Reductions of 4096 (Transformer-big FFN1's dgrad) run faster unsplit on 128x128 tiles since the
# K-outer loop stopped waiting for the next stage's DMA (65.8 vs 77.8 us; tools/linear_ab.py,
# profiles/linear_ab_r5.jsonl); the 33728-long logits reduction still gains (483 vs 576 us).
DGRAD_SPLITK_MAX_TILES = 192
DGRAD_SPLITK_MIN_RED = 8192


def _dgrad_splitk(dy2, w, dx, M: int, K: int, N: int) -> bool:
    tiles = ((M + 255) // 256) * ((K + 255) // 256)
    if tiles >= DGRAD_SPLITK_MAX_TILES or N < DGRAD_SPLITK_MIN_RED or K % 8 or M % 8 or N % 8:
        return False
    nkt = (N + 63) // 64
    splits = max(2, min(-(-256 // tiles), nkt // 16))
    ns = int(lib().gemm_splits(N, splits))
    if ns < 2:
        return False
    stride = ((M * K + 3) // 4) * 4
    ws = workspace(dx.device, ns * stride, slot="splitk")
    _gemm(dy2, w, ws, M, K, N, N, K, K, A_KIN, B_KOUT, EPI_F32, (256, 256), splits=splits, split_stride=stride)
    lib().splitk_reduce(ws, ns, stride, M * K, None, dx.view(-1), False, 1.0)
    return True


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, gw: torch.Tensor, accumulate: bool = False,
                 split_target: int | None = None) -> None:
    """gw[N,K] (f32) (+)= dy[M,N]^T @ x[M,K]. split_target: split-K fill target override (blocks)."""
    N = dy.shape[-1]
    K = x.shape[-1]
    dy2, x2 = dy.reshape(-1, N), x.reshape(-1, K)
    M = dy2.shape[0]
    if not on_gpu(dy):
        g = dy2.float().t() @ x2.float()
        if accumulate:
            gw.view(N, K).add_(g)
        else:
            gw.view(N, K).copy_(g)
        return
    if RECORD is not None:
        RECORD.append(("wgrad", (N, K, M), ()))
    tuned = tuning.wgrad_config(N, K, M) if (N % 8 == 0 and K % 8 == 0 and split_target is None) else None
    tile = tuned[0] if tuned else pick_tile(N, K, splits_ok=True, big_ok=True, K=M, split_target=split_target,
                                            g4=N % 8 == 0 and K % 8 == 0)
    tiles = ((N + tile[0] - 1) // tile[0]) * ((K + tile[1] - 1) // tile[1])
    if tuned is None and split_target is None and tile == (256, 256) and _wgrad_tail_split(dy2, x2, gw, N, K, M,
                                                                                           accumulate):
        return

    def run(C, splits, stride, beta):
        _gemm(dy2, x2, C, N, K, M, N, K, K, A_KOUT, B_KOUT, EPI_F32, tile, beta=beta, splits=splits,
              split_stride=stride)
    # beside the critical path (side stream): half the isolated-sweep fill, unless the model set
    # its own in-model target (BERT's 512: 11.25 ms/step, halved to 256: 11.41)
    div = SIDE_WGRAD_FILL_DIV if (_lib_mod.ON_SIDE_STREAM and split_target is None) else 1
    fs = tuned[1] if tuned else None
    if div > 1:
        fs = max(1, fs // div) if fs is not None else None
        split_target = TARGET_BLOCKS // div
    _f32_out_splitk(run, N, K, M, tiles, gw.view(-1), accumulate, dy.device, split_target=split_target,
                    force_splits=fs, slot=_lib_mod.WGRAD_SLOT)


# Weight gradients of a few whole rounds of 256x256 tiles plus a small tail (the tied-embedding
# gradient 33728 x 1024 = 528 tiles = 2 rounds + 16 tiles: unsplit, the 16-tile tail costs a third
# full-length round): the whole rounds run unsplit, the tail row-tiles split over the reduction
# into f32 slabs reduced into their rows of gw.
CHIP_BLOCKS = 256
TAIL_MAX_FRAC = 0.25


def _wgrad_tail_split(dy2, x2, gw, N: int, K: int, M: int, accumulate: bool) -> bool:
    tn, tm = -(-K // 256), -(-N // 256)
    tiles = tm * tn
    rounds, rem = divmod(tiles, CHIP_BLOCKS)
    if rounds < 1 or rem == 0 or rem > TAIL_MAX_FRAC * CHIP_BLOCKS or N % 8 or K % 8:
        return False
    rows_dp = (rounds * CHIP_BLOCKS) // tn  # whole row-tiles in the unsplit part
    n0 = rows_dp * 256
    if n0 == 0 or n0 >= N:  # no whole row-tile in the unsplit part (inputs wider than 65536): no zero-row launch
        return False
    nt = N - n0
    tail_tiles = -(-nt // 256) * tn
    nkt = (M + 63) // 64
    splits = max(2, min(CHIP_BLOCKS // tail_tiles, nkt // 8))
    ns = int(lib().gemm_splits(M, splits))
    if ns < 2:
        return False
    g = gw.view(N, K)
    # unsplit part: rows [0, n0)
    _gemm(dy2, x2, g, n0, K, M, N, K, K, A_KOUT, B_KOUT, EPI_F32, (256, 256), beta=1.0 if accumulate else 0.0)
    # tail rows [n0, N): A = dy columns n0.. (K-outer, lda = N), split over M into slabs
    stride = ((nt * K + 3) // 4) * 4
    ws = workspace(dy2.device, ns * stride, slot=_lib_mod.WGRAD_SLOT)
    _gemm(dy2.view(-1)[n0:], x2, ws, nt, K, M, N, K, K, A_KOUT, B_KOUT, EPI_F32, (256, 256), splits=splits,
          split_stride=stride)
    lib().splitk_reduce(ws, ns, stride, nt * K, g[n0:].reshape(-1), None, accumulate, 1.0)
    return True


def bias_grad(dy: torch.Tensor, gb: torch.Tensor, accumulate: bool = False) -> None:
    N = dy.shape[-1]
    dy2 = dy.reshape(-1, N)
    if not on_gpu(dy):
        g = dy2.float().sum(0)
        gb.add_(g) if accumulate else gb.copy_(g)
        return
    if not accumulate:
        gb.zero_()
    lib().colsum(dy2, dy2.shape[0], N, N, gb)


def matmul_tn(a: torch.Tensor, b: torch.Tensor, out_f32: torch.Tensor | None = None) -> torch.Tensor:
    """[M,N] = a[K,M]^T @ b[K,N]; f32 output."""
    K, M = a.shape
    N = b.shape[1]
    out = out_f32 if out_f32 is not None else torch.empty(M, N, dtype=torch.float32, device=a.device)
    if not on_gpu(a):
        out.copy_(a.float().t() @ b.float())
        return out
    tile = pick_tile(M, N, splits_ok=True, big_ok=True, K=K, g4=M % 8 == 0 and N % 8 == 0)
    tiles = ((M + tile[0] - 1) // tile[0]) * ((N + tile[1] - 1) // tile[1])

    def run(C, splits, stride, beta):
        _gemm(a, b, C, M, N, K, M, N, N, A_KOUT, B_KOUT, EPI_F32, tile, beta=beta, splits=splits, split_stride=stride)
    _f32_out_splitk(run, M, N, K, tiles, out.view(-1), False, a.device)
    return out


# =========================================================================== conv (NHWC)
def _ref_conv(x, w, g: ConvGeom):
    xn = x.float().permute(0, 3, 1, 2)
    wn = w.float().permute(0, 3, 1, 2)
    y = F.conv2d(xn, wn, stride=(g.sh, g.sw), padding=(g.ph, g.pw), dilation=(g.dh, g.dw))
    return y.permute(0, 2, 3, 1)


# Tile selection hooks for tools/conv_sweep.py: FORCE_TILE overrides every conv fwd / dgrad GEMM
# tile; RECORD (a list) collects (kind, geometry, flags) of every such call.
FORCE_TILE = None
RECORD = None


def _conv_tile(kind: str, g: ConvGeom, default, flags=()):
    if RECORD is not None:
        RECORD.append((kind, tuple(g.vec()), tuple(flags)))
    if FORCE_TILE is not None:
        return FORCE_TILE
    t = tuning.conv_tile(kind, tuple(g.vec()))
    return t if t is not None else default()


# ResNet stem (7x7/s2/p3, RGB padded to 8 channels -> 64) forward on the direct halo kernel
# (csrc/kernels/conv_stem.hip).
STEM = True


def stem_fwd_ok(g: ConvGeom, cin_used: int | None) -> bool:
    return bool(STEM and cin_used is not None and cin_used <= 4 and g.R == 7 and g.S == 7 and g.sh == 2
                and g.sw == 2 and g.ph == 3 and g.pw == 3 and g.dh == 1 and g.dw == 1 and g.C == 8 and g.K == 64
                and lib().stem_fwd_ok(g.N, g.H, g.W))


def conv_fwd(x: torch.Tensor, w: torch.Tensor, g: ConvGeom, stats: torch.Tensor | None = None,
             shards: int = 1, bias: torch.Tensor | None = None, act: str | None = None,
             cin_used: int | None = None) -> torch.Tensor:
    """y[N,P,Q,K] = act(conv(x[N,H,W,C], w[K,R,S,C]) + bias); optionally accumulates BN batch
    statistics (sum, sumsq per output channel) of the f32 result into stats[shards][2][K].
    cin_used: input channels that may be nonzero (the rest are zero padding)."""
    if not on_gpu(x):
        y = _ref_conv(x, w, g)
        if bias is not None:
            y = y + bias.float()
        y = act_ref(y, act)
        if stats is not None:
            yf = y.reshape(-1, g.K)
            stats.view(shards, 2, g.K)[0, 0] += yf.sum(0)
            stats.view(shards, 2, g.K)[0, 1] += (yf * yf).sum(0)
        return y.to(torch.bfloat16).contiguous()
    M = g.N * g.P * g.Q
    y = torch.empty(g.N, g.P, g.Q, g.K, dtype=torch.bfloat16, device=x.device)
    if bias is None and act is None and stem_fwd_ok(g, cin_used):
        lib().stem_fwd(x, w, y, stats, shards)
        return y
    tile = _conv_tile("fwd", g, lambda: pick_tile(M, g.K, big_ok=g.pointwise, K=g.R * g.S * g.C, mid_ok=g.pointwise,
                                                  g4=g.pointwise or g.C % 64 == 0 or (g.C % 8 == 0 and g.C < 64)),
                      (stats is not None, bias is not None, act is not None))
    if g.pointwise:
        _gemm(x, w, y, M, g.K, g.C, g.C, g.C, g.K, A_KIN, B_KIN, EPI_BF16, tile, stats=stats, shards=shards,
              bias=bias, act=ACT[act])
    else:
        Kd = g.R * g.S * g.C
        _gemm(x, w, y, M, g.K, Kd, 0, Kd, g.K, A_CONV_FWD, B_KIN, EPI_BF16, tile, stats=stats, shards=shards,
              conv=g.vec(), bias=bias, act=ACT[act])
    return y


def conv_weight_t(w: torch.Tensor, g: ConvGeom, out: torch.Tensor | None = None, flip: bool = False) -> torch.Tensor:
    """OHWI [K][R][S][C] -> [C][R][S][K] (dgrad B operand); flip: taps reversed,
    out[c][r][s][k] = w[k][R-1-r][S-1-s][c] (the stride-1 dgrad as a forward conv)."""
    if not on_gpu(w):
        t = w.flip(1, 2) if flip else w
        return t.permute(3, 1, 2, 0).contiguous()
    out = out if out is not None else torch.empty(g.C, g.R, g.S, g.K, dtype=torch.bfloat16, device=w.device)
    lib().transpose_arb(w, out, g.K, g.R * g.S, g.C, int(flip))
    return out


def dgrad_as_fwd_geom(g: ConvGeom) -> ConvGeom | None:
    """A stride-1, undilated conv's input gradient is a forward conv of dY with the flipped,
    transposed kernel: dx[n,h,w,c] = sum_{r,s,k} dy[n, h - (R-1-ph) + r', w - (S-1-pw) + s', k]
    * w[k][R-1-r'][S-1-s'][c]. Returns that forward conv's geometry (input dY [N,P,Q,K], Cout = C,
    pad R-1-ph), or None when the conv is not of that kind or the output size would differ."""
    if g.sh != 1 or g.sw != 1 or g.dh != 1 or g.dw != 1 or g.pointwise:
        return None
    if g.R - 1 - g.ph < 0 or g.S - 1 - g.pw < 0:
        return None
    f = ConvGeom(g.N, g.P, g.Q, g.K, g.C, g.R, g.S, 1, 1, g.R - 1 - g.ph, g.S - 1 - g.pw)
    return f if (f.P == g.H and f.Q == g.W) else None


# Stride-1 dgrads go through the LDS-DMA engine's conv-forward gather (its Cin = the conv's Cout
# must be a multiple of 64) for outputs of >= 128 channels (measured ResNet-50 step: 31.13 -> 30.81
# ms against the register-engine gather).
DGRAD_AS_FWD = True
# 64-channel dx: the 2-wave 128x64 BN epilogue measured slower (0.28 vs 0.22 ms)
DGRAD_AS_FWD_MIN_C = 128
# 3x3 / stride-1 / pad-1 convs of ResNet stage 1 (56x56x64) run on the halo-tile direct conv
# (csrc/kernels/conv_halo.hip; the C++ g4 launcher picks it for these shapes), forward and -- as a
# forward conv over dY -- dgrad. TFK_HALO=0 restores the implicit-GEMM gather; TFK_HALO=2 also
# routes stage 2 (28x28x128, measured level with the gather).
HALO = int(os.environ.get("TFK_HALO", "1"))


def halo_ok(f: ConvGeom) -> bool:
    """The forward conv f is one the halo kernel serves (mirrors tfk_halo_launch's eligibility)."""
    if not (HALO and G4_ENABLED and f.R == 3 and f.S == 3 and f.sh == 1 and f.sw == 1 and f.ph == 1
            and f.pw == 1 and f.dh == 1 and f.dw == 1 and f.P == f.H and f.Q == f.W and f.H % 4 == 0):
        return False
    return (f.W == 56 and f.C == 64 and f.K == 64) or (HALO >= 2 and f.W == 28 and f.C == 128 and f.K == 128)


# Strided-conv dgrad phases (BN-reduce epilogue with the phase out-map) as forward convs over dY on
# the LDS-DMA gather (needs the conv's Cout % 64 == 0).
PHASES_AS_FWD = True
# Non-pointwise weight gradients on the LDS-DMA engine's im2col gather (B_CONV_WGRAD, C % 8 == 0).
G4_WGRAD = True
# 3x3 / pad-1 / stride-1|2 weight gradients on the halo-tile direct kernel (csrc/kernels/conv_hwgrad.hip:
# one L2->LDS load of each band's input halo + dY for all nine taps, per-block f32 slabs + one
# splitk_reduce).
HWGRAD = True


def hwgrad_slabs(g: ConvGeom) -> int:
    """Slabs the halo weight-gradient kernel uses for conv g (0: shape not served)."""
    if not (HWGRAD and g.R == 3 and g.S == 3 and g.ph == 1 and g.pw == 1 and g.sh == g.sw and g.dh == 1
            and g.dw == 1 and g.C % 64 == 0 and g.K % 64 == 0):
        return 0
    return int(lib().hwgrad_slabs(g.N, g.H, g.W, g.P, g.Q, g.C, g.K, g.sh))


def _phases(g: ConvGeom):
    """Sub-pixel decomposition of a strided conv's dgrad: output phase (a, b) (rows h = a + sh*i)
    only receives the taps r = r0 + sh*i with r0 = (a + ph) % sh, and those read dY row
    i_h + (a + ph - r0)/sh - i -- a stride-1 dgrad with Rp x Sp taps on the phase grid. Returns
    [(a, b, Ha, Wb, r0, s0, Rp, Sp, ph', pw')]; None if some non-empty phase has no taps or the
    conv is dilated (-> gather path)."""
    if g.dh != 1 or g.dw != 1:
        return None
    out = []
    for a in range(g.sh):
        for b in range(g.sw):
            Ha, Wb = len(range(a, g.H, g.sh)), len(range(b, g.W, g.sw))
            if Ha == 0 or Wb == 0:
                continue
            r0, s0 = (a + g.ph) % g.sh, (b + g.pw) % g.sw
            Rp, Sp = len(range(r0, g.R, g.sh)), len(range(s0, g.S, g.sw))
            if Rp == 0 or Sp == 0:
                return None
            out.append((a, b, Ha, Wb, r0, s0, Rp, Sp, (a + g.ph - r0) // g.sh, (b + g.pw - s0) // g.sw))
    return out


def conv_dgrad(dy: torch.Tensor, w: torch.Tensor, g: ConvGeom, resid: torch.Tensor | None = None,
               wt: torch.Tensor | None = None, bnr=None, resid_stride: int = 1) -> torch.Tensor:
    """dx[N,H,W,C] = conv_transpose(dy[N,P,Q,K], w) (+ resid). bnr (ops.norm.BNReduce): also
    accumulate the BN-backward channel sums of the layer that produced x, from the final dx.
    resid_stride > 1 (pointwise convs with bnr): resid is [N, ceil(H/s), ceil(W/s), C] and is added
    on the stride-s lattice only -- the dgrad of a strided 1x1 projection shortcut computed densely
    on its own rows (no 3/4-zero gather), folded into the sibling conv's dgrad epilogue.
    Strided convs with bnr run as one stride-1 dgrad GEMM per output phase (``_phases``)."""
    if not on_gpu(dy):
        dyn = dy.float().permute(0, 3, 1, 2)
        wn = w.float().permute(0, 3, 1, 2)
        out_pad = (g.H - ((g.P - 1) * g.sh - 2 * g.ph + g.dh * (g.R - 1) + 1),
                   g.W - ((g.Q - 1) * g.sw - 2 * g.pw + g.dw * (g.S - 1) + 1))
        dx = F.conv_transpose2d(dyn, wn, stride=(g.sh, g.sw), padding=(g.ph, g.pw), output_padding=out_pad,
                                dilation=(g.dh, g.dw)).permute(0, 2, 3, 1)
        if resid is not None:
            if resid_stride > 1:
                full = torch.zeros_like(dx)
                full[:, ::resid_stride, ::resid_stride, :] = resid.float()
                resid = full
            dx = dx.to(torch.bfloat16).float() + resid.float()
        dx = dx.to(torch.bfloat16).contiguous()
        if bnr is not None:
            dz = bnr.reference_accumulate(dx)
            if bnr.premask:
                dx = dz.to(torch.bfloat16).reshape(dx.shape).contiguous()
        return dx
    M = g.N * g.H * g.W
    dx = torch.empty(g.N, g.H, g.W, g.C, dtype=torch.bfloat16, device=dy.device)
    def _default_tile():
        return pick_tile(M, g.C, big_ok=g.pointwise, K=g.K, mid_ok=g.pointwise, g4=g.pointwise and g.C % 8 == 0)
    flags = (resid is not None, bnr is not None, bnr is not None and bnr.a is not None,
             bnr is not None and bnr.y2 is not None, resid_stride)
    tile = _conv_tile("dgrad_pw", g, _default_tile, flags) if (g.pointwise and resid_stride == 1) else _default_tile()
    if resid_stride > 1:
        if not g.pointwise or bnr is None or resid is None:
            raise ValueError("resid_stride needs a pointwise conv, a resid and the fused BN reduction")
        s = resid_stride
        rmap = [0] * 8 + [g.H, g.W, -(-g.H // s), -(-g.W // s), s, s]
        _gemm(dy, w, dx, M, g.C, g.K, g.K, g.C, g.C, A_KIN, B_KOUT, EPI_BF16, tile, resid=resid, bnr=bnr,
              rowmap=rmap)
        return dx
    if g.pointwise:
        _gemm(dy, w, dx, M, g.C, g.K, g.K, g.C, g.C, A_KIN, B_KOUT, EPI_BF16, tile, resid=resid, bnr=bnr)
        return dx
    f = dgrad_as_fwd_geom(g) if (DGRAD_AS_FWD and G4_ENABLED and g.K % 64 == 0 and g.C % 8 == 0) else None
    if f is not None and g.C < DGRAD_AS_FWD_MIN_C and not halo_ok(f):
        f = None
    if f is not None:
        wf = conv_weight_t(w, g, flip=True)  # [C][R][S][K]: the forward conv's OHWI weight
        Kd = g.R * g.S * g.K
        _gemm(dy, wf, dx, M, g.C, Kd, 0, Kd, g.C, A_CONV_FWD, B_KIN, EPI_BF16,
              _conv_tile("dgrad_fwd", g, lambda: pick_tile(M, g.C, K=Kd, mid_ok=False, g4=True), flags),
              resid=resid, conv=f.vec(), bnr=bnr)
        return dx
    phases = _phases(g) if (bnr is not None and (g.sh > 1 or g.sw > 1)) else None
    if phases is not None:
        wt = wt if wt is not None else conv_weight_t(w, g)
        as_fwd = PHASES_AS_FWD and G4_ENABLED and g.K % 64 == 0
        for a, b, Ha, Wb, r0, s0, Rp, Sp, php, pwp in phases:
            wp = wt[:, r0::g.sh, s0::g.sw, :]  # [C][Rp][Sp][K] sub-kernel (weights only)
            Mp, Kd = g.N * Ha * Wb, Rp * Sp * g.K
            rmap = [Ha, Wb, g.H, g.W, g.sh, g.sw, a, b] + [0] * 6
            if as_fwd:
                # the phase's stride-1 dgrad as a forward conv over dY (flipped taps, pad Rp-1-php)
                # on the LDS-DMA gather; GEMM rows walk the phase grid, the out-map scatters them
                conv = [g.N, g.P, g.Q, g.K, Ha, Wb, g.C, Rp, Sp, 1, 1, Rp - 1 - php, Sp - 1 - pwp, 1, 1]
                _gemm(dy, wp.flip(1, 2).contiguous(), dx, Mp, g.C, Kd, 0, Kd, g.C, A_CONV_FWD, B_KIN, EPI_BF16,
                      pick_tile(Mp, g.C, K=Kd, mid_ok=False, g4=True), resid=resid, conv=conv, bnr=bnr, rowmap=rmap)
            else:
                conv = [g.N, Ha, Wb, g.C, g.P, g.Q, g.K, Rp, Sp, 1, 1, php, pwp, 1, 1]
                _gemm(dy, wp.contiguous(), dx, Mp, g.C, Kd, 0, Kd, g.C, A_CONV_DGRAD, B_KIN, EPI_BF16,
                      pick_tile(Mp, g.C, K=Kd, mid_ok=False), resid=resid, conv=conv, bnr=bnr, rowmap=rmap)
        return dx
    if g.R == 1 and g.S == 1:
        # strided 1x1: B(n=c, k=co) = W[co][c] is K-outer with ldb = C; gather handles the stride
        _gemm(dy, w, dx, M, g.C, g.K, 0, g.C, g.C, A_CONV_DGRAD, B_KOUT, EPI_BF16, tile, resid=resid,
              conv=g.vec(), bnr=bnr)
    else:
        wt = wt if wt is not None else conv_weight_t(w, g)
        Kd = g.R * g.S * g.K
        _gemm(dy, wt, dx, M, g.C, Kd, 0, Kd, g.C, A_CONV_DGRAD, B_KIN, EPI_BF16, tile, resid=resid, conv=g.vec(),
              bnr=bnr)
    return dx


def stem_wgrad_slabs(g: ConvGeom, cin_used: int | None) -> int:
    """Slabs of the direct stem weight-gradient kernel (ResNet conv1: 7x7/s2/p3, 8-channel padded
    input of which at most 4 are nonzero, 64 outputs); 0 when the conv is not of that kind."""
    if not (HWGRAD and cin_used is not None and cin_used <= 4 and g.R == 7 and g.S == 7 and g.sh == 2
            and g.sw == 2 and g.ph == 3 and g.pw == 3 and g.dh == 1 and g.dw == 1 and g.C == 8 and g.K == 64):
        return 0
    return int(lib().stem_wgrad_slabs(g.N, g.H, g.W))


def conv_wgrad(dy: torch.Tensor, x: torch.Tensor, g: ConvGeom, gw: torch.Tensor, accumulate: bool = False,
               splits: int | None = None, cin_used: int | None = None) -> None:
    """gw[K][R][S][C] (f32) (+)= sum over (n,p,q) dy[n,p,q,k] * x[n, p*sh-ph+r, q*sw-pw+s, c].
    cin_used: input channels that may be nonzero (the rest are zero padding, whose gradient is 0)."""
    explicit = splits is not None
    Nn = g.R * g.S * g.C
    Kp = g.N * g.P * g.Q
    if not on_gpu(dy):
        xn = x.float().permute(0, 3, 1, 2)
        dyn = dy.float().permute(0, 3, 1, 2)
        gwt = torch.nn.grad.conv2d_weight(xn, (g.K, g.C, g.R, g.S), dyn, stride=(g.sh, g.sw), padding=(g.ph, g.pw),
                                          dilation=(g.dh, g.dw)).permute(0, 2, 3, 1).reshape(g.K, Nn)
        v = gw.view(g.K, Nn)
        v.add_(gwt) if accumulate else v.copy_(gwt)
        return
    ns = stem_wgrad_slabs(g, cin_used) if splits is None else 0
    if ns > 0:
        n = g.K * Nn
        ws = workspace(dy.device, ns * n, slot=_lib_mod.WGRAD_SLOT)
        lib().stem_wgrad(x, dy, ws, g.N, g.H, g.W, ns)
        lib().splitk_reduce(ws, ns, n, n, gw.view(-1), None, accumulate, 1.0)
        return
    ns = hwgrad_slabs(g) if splits is None else 0
    if ns > 0:
        n = g.K * Nn
        ws = workspace(dy.device, ns * n, slot=_lib_mod.WGRAD_SLOT)
        lib().hwgrad(x, dy, ws, g.N, g.H, g.W, g.P, g.Q, g.C, g.K, g.sh, ns)
        lib().splitk_reduce(ws, ns, n, n, gw.view(-1), None, accumulate, 1.0)
        return
    # measured table first (pointwise = dense GEMM shapes, tools/wgrad_sweep.py), else the model
    if RECORD is not None and g.pointwise:
        RECORD.append(("wgrad", (g.K, Nn, Kp), ()))
    tuned = tuning.wgrad_config(g.K, Nn, Kp) if (g.pointwise and g.K % 8 == 0 and g.C % 8 == 0) else None
    if splits is None and tuned is not None:
        tile, splits = tuned
    else:
        tile = pick_tile(g.K, Nn, splits_ok=True, big_ok=g.pointwise, K=Kp,
                         wide_ok=WIDE_WGRAD and not g.pointwise and g.C <= WIDE_WGRAD_MAX_C,
                         g4=(G4_WGRAD or g.pointwise) and g.K % 8 == 0 and g.C % 8 == 0,
                         narrow_ok=G4_WGRAD and not g.pointwise, rect_ok=g.pointwise)
    tiles = ((g.K + tile[0] - 1) // tile[0]) * ((Nn + tile[1] - 1) // tile[1])

    def run(C, sp, stride, beta):
        if g.pointwise:
            _gemm(dy, x, C, g.K, Nn, Kp, g.K, g.C, Nn, A_KOUT, B_KOUT, EPI_F32, tile, beta=beta, splits=sp,
                  split_stride=stride)
        else:
            _gemm(dy, x, C, g.K, Nn, Kp, g.K, 0, Nn, A_KOUT, B_CONV_WGRAD, EPI_F32, tile, beta=beta, splits=sp,
                  split_stride=stride, conv=g.vec())
    # own slab workspace: conv weight gradients may run on the side stream (runtime/streams.py)
    div = SIDE_WGRAD_FILL_DIV if (_lib_mod.ON_SIDE_STREAM and not explicit) else 1
    if div > 1 and splits is not None:
        splits = max(1, splits // div)
    _f32_out_splitk(run, g.K, Nn, Kp, tiles, gw.view(-1), accumulate, dy.device, force_splits=splits,
                    slot=_lib_mod.WGRAD_SLOT, split_target=TARGET_BLOCKS // div)
