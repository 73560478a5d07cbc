"""Executor layers with explicit forward/backward on the tfk kernel library.

No torch autograd in the hot path: each layer saves exactly what its backward needs, writes its
weight gradients straight into the flat arena (f32) and signals readiness to the data-parallel
strategy, so all-reduce of early buckets overlaps the rest of backward.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import gemm as G
from ..ops import norm as BN
from ..ops import transformer as TR
from . import streams
from .arena import ParamArena, ParamSpec


def _ohwi_to_hwio(a: np.ndarray, cin_real: int | None = None) -> np.ndarray:
    a = np.transpose(a, (1, 2, 3, 0))  # [R,S,C,K]
    return a[:, :, :cin_real, :] if cin_real is not None else a


def _hwio_to_ohwi(a: np.ndarray, cin_pad: int | None = None) -> np.ndarray:
    if cin_pad is not None and a.shape[2] < cin_pad:
        pad = np.zeros(a.shape[:2] + (cin_pad - a.shape[2], a.shape[3]), dtype=a.dtype)
        a = np.concatenate([a, pad], axis=2)
    return np.ascontiguousarray(np.transpose(a, (3, 0, 1, 2)))


def linear_forward(x, w, b, fp8: bool, **kw):
    """bf16 GEMM, or the MX-fp8 block-scaled MFMA GEMM when fp8 and K % 128 == 0 (which also
    leaves MX(x^T) / MX(w^T) for this step's backward: ops.fp8.save_t)."""
    if fp8 and x.shape[-1] % 128 == 0:
        from ..ops.fp8 import linear_fwd_mx
        return linear_fwd_mx(x, w, b, save=True, **kw)
    kw.pop("mx_out", None)
    kw.pop("mx_skip_c", None)
    return G.linear_fwd(x, w, b, **kw)


def fp8_dy(dy, K: int, fp8: bool):
    """The backward's MX operands of dy [M, N] for a layer with K inputs: (MX(dy) for dgrad,
    MX(dy^T) for wgrad), both from one read when both GEMMs run in fp8; None where a GEMM stays
    bf16 (or fp8 is off)."""
    if not fp8:
        return None, None
    from ..ops.fp8 import mx_backward_ok, mx_quantize_dual
    M, N = dy.shape
    dg, wg = mx_backward_ok(M, N, K)
    from ..ops.fp8 import cached_dual
    c = cached_dual(dy)  # the dgrad that produced dy already wrote its MX copies
    if dg and wg:
        return c if c is not None else mx_quantize_dual(dy)
    if dg and c is not None:
        return c[0], None
    return None, None


def linear_wgrad(dy, x, gw, fp8: bool, accumulate: bool = False, split_target=None, dyt=None):
    """Weight gradient: MX-fp8 when fp8 and the token count tiles (M % 128), else bf16 split-K."""
    if fp8:
        from ..ops.fp8 import linear_wgrad_mx, mx_backward_ok
        if mx_backward_ok(dy.shape[0], dy.shape[1], x.shape[1])[1]:
            return linear_wgrad_mx(dy, x, gw, accumulate=accumulate, dyt=dyt)
        from ..ops.fp8 import check_stored
        check_stored(dy, x)  # the bf16 GEMM below reads bf16 values: none may be an MX-only output
    return G.linear_wgrad(dy, x, gw, accumulate=accumulate, split_target=split_target)


def _mx_keep(dyt) -> tuple:
    """The tensors of an MX operand (q, scales) a deferred weight gradient reads (kept alive by
    runtime.streams until the join)."""
    return tuple(t for t in (dyt or ()) if isinstance(t, torch.Tensor))


def linear_dgrad(dy, w, fp8: bool, drop_p: float = 0.0, drop_seed: int = 0, dyq=None, **kw):
    """Input gradient: MX-fp8 when fp8 and the output width tiles (N % 128), else bf16; either way
    the input-dropout backward runs in the GEMM epilogue."""
    if fp8:
        from ..ops.fp8 import linear_dgrad_mx, mx_backward_ok
        if mx_backward_ok(dy.shape[0], dy.shape[1], w.shape[1])[0]:
            return linear_dgrad_mx(dy, w, dyq=dyq, drop_p=drop_p, drop_seed=drop_seed, **kw)
        from ..ops.fp8 import check_stored
        check_stored(dy)
    kw.pop("mx_out", None)
    kw.pop("mx_skip_c", None)
    return G.linear_dgrad(dy, w, drop_p=drop_p, drop_seed=drop_seed, **kw)


class Conv2d:
    """NHWC conv, OHWI weight. TF variable: <name>/kernel in HWIO."""

    def __init__(self, arena: ParamArena, name: str, cin: int, cout: int, k: int, stride: int = 1, pad: int | None = None,
                 cin_real: int | None = None, cout_real: int | None = None, bias: bool = False):
        """cin_real/cout_real < cin/cout: channels padded to multiples of 8 for 16-B NHWC vectors
        (e.g. RGB stem, LeNet's 1->6 conv); padded weights start and stay exactly zero, and the
        checkpoint holds only the real [k, k, cin_real, cout_real] kernel."""
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.cin_real = cin_real if cin_real is not None else cin
        self.pad = (k - 1) // 2 if pad is None else pad
        real = cin_real if cin_real is not None else cin
        oreal = cout_real if cout_real is not None else cout
        post = None
        if real != cin or oreal != cout:
            def post(t, real=real, oreal=oreal):
                t[..., real:] = 0
                t[oreal:] = 0
                return t

        def to_tf(a, real=real, oreal=oreal):
            return _ohwi_to_hwio(a, real)[..., :oreal]

        def from_tf(a, c=cin, co=cout):
            if a.shape[3] < co:
                a = np.concatenate([a, np.zeros(a.shape[:3] + (co - a.shape[3],), dtype=a.dtype)], axis=3)
            return _hwio_to_ohwi(a, c)
        self.w = arena.add(ParamSpec(
            f"{name}/kernel", (cout, k, k, cin), init="he_normal", fan_in=k * k * real, fan_out=k * k * oreal,
            to_tf=to_tf, from_tf=from_tf, tf_shape=(k, k, real, oreal), post_init=post))
        self.b = None
        if bias:
            self.b = arena.add(ParamSpec(f"{name}/bias", (cout,), init="zeros", decay=False,
                                         to_tf=lambda a, o=oreal: a[:o],
                                         from_tf=lambda a, co=cout: np.concatenate([a, np.zeros(co - a.shape[0], a.dtype)])))
        self.arena = arena

    def geom(self, x_shape) -> G.ConvGeom:
        N, H, W, C = x_shape
        assert C == self.cin, f"conv expects {self.cin} input channels, got {C}"
        return G.ConvGeom(N, H, W, C, self.cout, self.k, self.k, self.stride, self.stride, self.pad, self.pad)

    def forward(self, x, stats: BN.BNState | None = None, act: str | None = None):
        g = self.geom(x.shape)
        return G.conv_fwd(x, self.w.compute, g, stats.stats if stats else None, stats.shards if stats else 1,
                          bias=self.b.master if self.b is not None else None, act=act, cin_used=self.cin_real)

    def backward(self, dy, x, need_dx: bool = True, resid=None, bnr=None, resid_stride: int = 1):
        g = self.geom(x.shape)
        streams.run_wgrad(lambda: G.conv_wgrad(dy, x, g, self.w.grad, cin_used=self.cin_real), dy, x, deferrable=True)
        if self.b is not None:
            G.bias_grad(dy, self.b.grad)
            self.arena.grad_ready(self.w, self.b)
        else:
            self.arena.grad_ready(self.w)
        if not need_dx:
            return None
        return G.conv_dgrad(dy, self.w.compute, g, resid=resid, bnr=bnr, resid_stride=resid_stride)

    def backward_lattice(self, dy, x):
        """Strided 1x1 conv (projection shortcut): weight gradient + the input gradient on the
        stride lattice only, as a dense [N, P, Q, C] GEMM (every other input position gets zero).
        The caller folds it into a sibling dgrad with ``resid_stride=stride``."""
        g = self.geom(x.shape)
        if self.k != 1 or self.pad != 0 or self.b is not None:
            raise ValueError("backward_lattice is for bias-free 1x1 convs")
        self.wgrad(dy, x)
        return self.lattice_dgrad(dy, x)

    def wgrad(self, dy, x):
        """Weight gradient only (side stream when enabled) + readiness notification."""
        g = self.geom(x.shape)
        streams.run_wgrad(lambda: G.conv_wgrad(dy, x, g, self.w.grad, cin_used=self.cin_real), dy, x, deferrable=True)
        self.arena.grad_ready(self.w)

    def lattice_dgrad(self, dy, x):
        """The input gradient of backward_lattice only (no weight gradient, no hooks)."""
        g = self.geom(x.shape)
        w2 = self.w.compute.view(self.cout, self.cin)
        return G.linear_dgrad(dy.reshape(-1, self.cout), w2).view(g.N, g.P, g.Q, g.C)


class BatchNorm:
    """Training-mode BN; TF variables <name>/{gamma,beta,moving_mean,moving_variance}."""

    def __init__(self, arena: ParamArena, name: str, C: int, eps: float = 1e-5, momentum: float = 0.1,
                 zero_gamma: bool = False):
        self.C, self.eps, self.momentum = C, eps, momentum
        self.gamma = arena.add(ParamSpec(f"{name}/gamma", (C,), init="zeros" if zero_gamma else "ones", decay=False))
        self.beta = arena.add(ParamSpec(f"{name}/beta", (C,), init="zeros", decay=False))
        self.run_mean = arena.add_buffer(f"{name}/moving_mean", torch.zeros(C))
        self.run_var = arena.add_buffer(f"{name}/moving_variance", torch.ones(C))
        self.arena = arena
        self.st: BN.BNState | None = None
        self.training = True

    def state(self, device) -> BN.BNState:
        if self.st is None or self.st.mean.device != torch.device(device):
            self.st = BN.BNState(self.C, device)
        return self.st

    def finalize(self, count: int, defer: bool = False) -> None:
        """defer: fold the finalize into the next bn_apply on this layer's state (pooled GPU states)."""
        BN.bn_finalize(self.st, float(count), self.gamma.master, self.beta.master, self.eps, self.momentum,
                       self.run_mean if self.training else None, self.run_var if self.training else None, defer=defer)

    def use_running_stats(self) -> None:
        """Inference: scale/shift from the moving statistics."""
        st = self.st
        inv = torch.rsqrt(self.run_var + self.eps)
        st.mean.copy_(self.run_mean); st.invstd.copy_(inv)
        st.scale.copy_(self.gamma.master * inv)
        st.shift.copy_(self.beta.master - self.run_mean * self.gamma.master * inv)


class Linear:
    """y = x W^T + b; W stored [out][in] (TF kernel is [in][out])."""

    def __init__(self, arena: ParamArena, name: str, fin: int, fout: int, bias: bool = True, init: str = "xavier_uniform",
                 std: float = 0.02, kernel_name: str = "kernel"):
        self.fin, self.fout = fin, fout
        self.w = arena.add(ParamSpec(f"{name}/{kernel_name}", (fout, fin), init=init, std=std, fan_in=fin, fan_out=fout,
                                     to_tf=lambda a: np.ascontiguousarray(a.T),
                                     from_tf=lambda a: np.ascontiguousarray(a.T), tf_shape=(fin, fout)))
        self.b = arena.add(ParamSpec(f"{name}/bias", (fout,), init="zeros", decay=False)) if bias else None
        self.arena = arena
        self.fp8 = False  # forward, dgrad and wgrad GEMMs in MX-fp8 (ops.fp8)
        self.split_target = None  # weight-gradient split-K fill target override (ops.gemm.pick_splits)

    def forward(self, x, act=None, resid=None, aux=None, drop_p: float = 0.0, drop_seed: int = 0,
                mx_out: bool = False, mx_skip_c: bool = False):
        """mx_out / mx_skip_c (fp8): the epilogue also emits MX(y), MX(y^T) for the next fp8 GEMM on y
        (and skips the bf16 y when every consumer is such a GEMM; ops.fp8.linear_fwd_mx)."""
        kw = {"mx_out": mx_out, "mx_skip_c": mx_skip_c} if mx_out else {}
        return linear_forward(x, self.w.compute, self.b.master if self.b else None, self.fp8, act=act, resid=resid,
                              aux=aux, drop_p=drop_p, drop_seed=drop_seed, **kw)

    def bias_sink(self):
        """The f32 bias-gradient view a producer kernel may accumulate into (pre-zeroed this step), or None."""
        return self.b.grad if self.b is not None and self.arena.prezeroed else None

    def backward(self, dy, x, need_dx: bool = True, resid=None, accumulate: bool = False, dact_src=None,
                 dact=None, drop_p: float = 0.0, drop_seed: int = 0, mx_dx: bool = False, bias_done: bool = False,
                 dx_bias=None, mx_dx_only: bool = False):
        """dy: gradient of this layer's (pre-dropout, post-activation-backward) output. drop_p/drop_seed:
        a forward dropout on this layer's input, whose backward is fused into the dgrad epilogue.
        mx_dx (fp8): the dgrad epilogue also emits MX(dx), MX(dx^T) for the producer's fp8 backward
        (mx_dx_only: and no bf16 dx). dx_bias: the producer layer's bias gradient (its bias_sink()),
        accumulated from dx's column sums in the dgrad epilogue."""
        dyq, dyt = fp8_dy(dy.reshape(-1, dy.shape[-1]), self.fin, self.fp8 and need_dx)

        def wgrad():
            linear_wgrad(dy, x, self.w.grad, self.fp8, accumulate=accumulate, split_target=self.split_target, dyt=dyt)
            if self.b is not None and not bias_done:
                G.bias_grad(dy, self.b.grad, accumulate=accumulate or self.arena.prezeroed)
        # on a side stream under capture (runtime/streams.py), concurrent with the input-gradient chain;
        # MX-fp8 ones are forked at once (their operands come from per-step caches), bf16 ones queue
        # for the layer's flush()
        streams.run_wgrad(wgrad, dy, x, *_mx_keep(dyt), deferrable=not self.fp8)
        if self.b is not None:
            self.arena.grad_ready(self.w, self.b)
        else:
            self.arena.grad_ready(self.w)
        if not need_dx:
            return None
        kw = {"mx_out": True, "mx_skip_c": mx_dx_only} if mx_dx else {}
        if dx_bias is not None:
            kw["colsum"] = dx_bias
        return linear_dgrad(dy, self.w.compute, self.fp8, resid=resid, dact_src=dact_src, dact=dact, drop_p=drop_p,
                            drop_seed=drop_seed, dyq=dyq, **kw)


class FusedLinear:
    """Several TF dense layers sharing one input, run as ONE GEMM (e.g. BERT's query/key/value ->
    a [3W, W] weight, 3x fewer launches and a 3x wider N for MFMA occupancy). Each part keeps its
    own TF variables (<name>/kernel [in, out], <name>/bias); registration back-to-back makes
    the arena place them contiguously (in reverse registration order: see ``cols``)."""

    def __init__(self, arena: ParamArena, names: list[str], fin: int, fout: int, init: str = "trunc_normal",
                 std: float = 0.02, bias: bool = True):
        self.arena, self.fin, self.fout, self.names = arena, fin, fout, names
        self.parts = [Linear(arena, n, fin, fout, init=init, std=std, bias=bias) for n in names]
        self.has_bias = bias
        self.fp8 = False
        self._views = None

    def _build(self):
        a = self.arena
        lo, hi = a.span([p.w for p in self.parts])
        order = sorted(range(len(self.parts)), key=lambda i: self.parts[i].w.offset)
        self.cols = {self.names[i]: k * self.fout for k, i in enumerate(order)}
        n = len(self.parts) * self.fout
        bm = bg = None
        if self.has_bias:
            blo, bhi = a.span([p.b for p in self.parts])
            if sorted(range(len(self.parts)), key=lambda i: self.parts[i].b.offset) != order:
                raise ValueError("fused bias order differs from kernel order")
            bm, bg = a.master[blo:bhi], a.grad[blo:bhi]
        self._views = (a.compute[lo:hi].view(n, self.fin), a.grad[lo:hi].view(n, self.fin), bm, bg)

    def views(self):
        if self._views is None:
            self._build()
        return self._views

    def col(self, name: str) -> int:
        self.views()
        return self.cols[name]

    def forward(self, x, act=None):
        w, _, b, _ = self.views()
        return linear_forward(x, w, b, self.fp8, act=act)

    def backward(self, dy, x, need_dx: bool = True, resid=None):
        w, gw, _, gb = self.views()
        dyq, dyt = fp8_dy(dy.reshape(-1, dy.shape[-1]), self.fin, self.fp8 and need_dx)

        def wgrad():
            linear_wgrad(dy, x, gw, self.fp8, split_target=getattr(self, "split_target", None), dyt=dyt)
            if gb is not None:
                G.bias_grad(dy, gb, accumulate=self.arena.prezeroed)
        streams.run_wgrad(wgrad, dy, x, *_mx_keep(dyt), deferrable=not self.fp8)
        self.arena.grad_ready(*[p.w for p in self.parts], *[p.b for p in self.parts if p.b is not None])
        if not need_dx:
            return None
        return linear_dgrad(dy, w, self.fp8, resid=resid, dyq=dyq)


def fp8_weight(lin) -> torch.Tensor:
    """The bf16 [out, in] weight a Linear / FusedLinear feeds its (MX-fp8) GEMMs."""
    return lin.views()[0] if isinstance(lin, FusedLinear) else lin.w.compute


def weight_quantizer(model, lins: list, extra: list | None = None):
    """The model's per-step grouped MX quantizer of its fp8 linear weights (built once; reset by
    ``model._wq = None`` when the arena moves)."""
    if getattr(model, "_wq", None) is None:
        from ..ops.fp8 import GroupQuantizer
        model._wq = GroupQuantizer([fp8_weight(l) for l in lins] + list(extra or []))
    return model._wq


def _mx_producers() -> bool:
    """models.transformer.MX_PRODUCERS (TFK_FP8_MX_PRODUCERS): producers emit fp8 consumers' MX operands."""
    import sys
    m = sys.modules.get("tensorflow_k8s_amd.models.transformer")
    return bool(getattr(m, "MX_PRODUCERS", True)) if m is not None else True


class LayerNorm:
    """TF variables <name>/gamma, <name>/beta (f32, no weight decay)."""

    def __init__(self, arena: ParamArena, name: str, W: int, eps: float = 1e-12, names=("gamma", "beta")):
        self.W, self.eps, self.arena = W, eps, arena
        self.gamma = arena.add(ParamSpec(f"{name}/{names[0]}", (W,), init="ones", decay=False))
        self.beta = arena.add(ParamSpec(f"{name}/{names[1]}", (W,), init="zeros", decay=False))

    def forward(self, x, mx_out: bool = False):
        """mx_out (fp8 training): y feeds only MX-fp8 GEMMs -- emit MX(y), MX(y^T), no bf16 y."""
        from ..ops import fp8 as F8
        # the bf16 y stays when the consumer's weight gradient reads it in bf16 (F8.MX_WGRAD off)
        y, mu, rs = TR.layernorm_fwd(x, self.gamma.master, self.beta.master, self.eps, mx_out=mx_out,
                                     skip_y=mx_out and F8.MX_WGRAD)
        return y, (mu, rs)

    def backward(self, dy, x, stats, dres=None, drop=None, consumer=None):
        """dx = LN'(x)^T dy (+ dres: gradient arriving through a residual connection). drop=(p, seed):
        returns (dx, dropout(dx, p, seed)) from one kernel (the consumer's dropout backward).
        consumer: the Linear whose output gradient this is -- its bias gradient is reduced here
        (``consumer.backward(..., bias_done=True)`` then skips its column-sum pass)."""
        mu, rs = stats
        if drop is not None and len(drop) > 2:  # (p, seed, consumer Linear or None)
            drop, consumer = drop[:2], drop[2] if consumer is None else consumer
        dbias = consumer.bias_sink() if consumer is not None else None
        # an fp8 consumer whose gradient rows tile the MX-fp8 K-tile takes MX operands from this kernel
        rows = dy.numel() // dy.shape[-1]
        mx = consumer is not None and getattr(consumer, "fp8", False) and rows % 128 == 0 and _mx_producers()
        dx = TR.layernorm_bwd(dy, x, self.gamma.master, mu, rs, self.gamma.grad, self.beta.grad, dres=dres,
                              accumulate=self.arena.prezeroed, drop=drop, dbias=dbias, mx_out=mx)
        self.arena.grad_ready(self.gamma, self.beta)
        return dx


def _pad_rows(rows: int, to: int = 128) -> int:
    return (rows + to - 1) // to * to


class Embedding:
    """Token embedding table [V, W] stored with V padded to a multiple of 128 rows (padding rows
    stay zero; the TF variable is the real [V, W] table). Also used as the tied output
    projection (logits = h @ table^T over the padded vocab, masked to V by the loss); 128 = one
    MX-fp8 K-tile, so that projection's input gradient -- a reduction over the padded vocab --
    runs on the fp8 GEMM as well."""

    def __init__(self, arena: ParamArena, name: str, V: int, W: int, std: float = 0.02, decay: bool = True):
        self.V, self.Vp, self.W = V, _pad_rows(V), W

        def post(t, V=V):
            t[V:] = 0
            return t
        self.table = arena.add(ParamSpec(name, (self.Vp, W), init="trunc_normal", std=std, decay=decay,
                                         post_init=post, tf_shape=(V, W), to_tf=lambda a, V=V: a[:V],
                                         from_tf=lambda a, Vp=self.Vp: np.concatenate(
                                             [a, np.zeros((Vp - a.shape[0], a.shape[1]), a.dtype)])))
