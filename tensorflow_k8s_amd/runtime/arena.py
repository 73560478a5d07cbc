"""Flat parameter arena: every parameter of a model lives in ONE f32 master buffer, ONE bf16
compute copy, ONE f32 gradient buffer and one buffer per optimizer slot.

Why (MI355X-first): the fused optimizer is a single launch over the whole arena (no
multi-tensor-apply lists), data-parallel gradient buckets are plain contiguous slices of the grad
buffer (one RCCL call per bucket, no flatten/unflatten copies), and checkpoint save/restore is a
handful of large D2H copies. Layout: weight-decayed params first, then the no-decay group
(BN gamma/beta, biases, LayerNorm); inside each group params are placed in REVERSE registration
(=forward) order so backward fills the gradient buffer front-to-back and buckets complete in order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch


@dataclass
class ParamSpec:
    name: str                      # TF-style variable name, e.g. "resnet50/conv1/kernel"
    shape: tuple                   # storage layout shape (e.g. OHWI for conv kernels)
    init: str = "zeros"            # zeros | ones | normal | he_normal | xavier_uniform | uniform
    std: float = 0.02
    fan_in: int = 1
    fan_out: int = 1
    decay: bool = True
    # storage <-> TF checkpoint layout converters (numpy); identity by default
    to_tf: Callable | None = None
    from_tf: Callable | None = None
    tf_shape: tuple | None = None
    post_init: Callable | None = None  # e.g. zero the padded input channels of a stem conv


@dataclass
class Param:
    spec: ParamSpec
    index: int
    offset: int = 0
    master: torch.Tensor | None = None   # f32 view
    compute: torch.Tensor | None = None  # bf16 view (what kernels read)
    grad: torch.Tensor | None = None     # f32 view

    @property
    def name(self):
        return self.spec.name

    @property
    def numel(self):
        return int(np.prod(self.spec.shape)) if self.spec.shape else 1


@dataclass
class BufferSpec:
    """Non-trainable state saved in checkpoints (BN moving statistics, global_step...)."""
    name: str
    tensor: torch.Tensor
    to_tf: Callable | None = None


ALIGN = 64  # elements; keeps every param view 256-B aligned (16-B vector loads, 128-B lines)


class ParamArena:
    def __init__(self):
        self.params: list[Param] = []
        self.buffers: list[BufferSpec] = []
        self.master = self.compute = self.grad = None
        self.slots: dict[str, torch.Tensor] = {}
        self.n_decay = 0  # elements in the decay region (region [0, n_decay))
        self.numel = 0
        self._ready_cbs: list[Callable] = []
        self.device = None
        # True while a step runs whose no-decay gradients (biases, LayerNorm/BN gamma+beta) were
        # zeroed in ONE fill up front (zero_nodecay_grads): their atomic-accumulating kernels then
        # skip their own per-tensor zero fills (BERT-base: ~80 fill launches per step -> 1)
        self.prezeroed = False

    # ------------------------------------------------------------------ construction
    def add(self, spec: ParamSpec) -> Param:
        if any(p.spec.name == spec.name for p in self.params):
            raise ValueError(f"duplicate parameter name {spec.name}")
        p = Param(spec=spec, index=len(self.params))
        self.params.append(p)
        return p

    def add_buffer(self, name: str, tensor: torch.Tensor, to_tf=None) -> torch.Tensor:
        self.buffers.append(BufferSpec(name, tensor, to_tf))
        return tensor

    def finalize(self, device, seed: int = 1234) -> "ParamArena":
        self.device = torch.device(device)
        decay = [p for p in reversed(self.params) if p.spec.decay]
        nodecay = [p for p in reversed(self.params) if not p.spec.decay]
        off = 0
        for grp in (decay, nodecay):
            for p in grp:
                p.offset = off
                off += ((p.numel + ALIGN - 1) // ALIGN) * ALIGN
            if grp is decay:
                self.n_decay = off
        self.numel = max(off, ALIGN)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.compute = torch.zeros(self.numel, dtype=torch.bfloat16, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        gen = torch.Generator().manual_seed(seed)
        host = torch.zeros(self.numel, dtype=torch.float32)
        for p in self.params:
            host[p.offset:p.offset + p.numel] = _init_values(p.spec, gen).reshape(-1)
        self.master.copy_(host)
        self.compute.copy_(self.master)
        for p in self.params:
            sl = slice(p.offset, p.offset + p.numel)
            p.master = self.master[sl].view(p.spec.shape)
            p.compute = self.compute[sl].view(p.spec.shape)
            p.grad = self.grad[sl].view(p.spec.shape)
        for b in self.buffers:
            b.tensor.data = b.tensor.data.to(self.device)
        return self

    def slot(self, name: str) -> torch.Tensor:
        if name not in self.slots:
            self.slots[name] = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        return self.slots[name]

    def refresh_compute(self) -> None:
        """master (f32) -> compute (bf16), e.g. after a checkpoint restore or a broadcast."""
        from ..ops.optim import cast_f32_bf16
        cast_f32_bf16(self.master, self.compute)

    # ------------------------------------------------------------------ grad readiness (DP overlap)
    def on_grad_ready(self, cb: Callable) -> None:
        self._ready_cbs.append(cb)

    def clear_grad_ready(self) -> None:
        self._ready_cbs.clear()

    def grad_ready(self, *params: Param) -> None:
        for cb in self._ready_cbs:
            for p in params:
                cb(p)

    def zero_nodecay_grads(self) -> None:
        lo, hi = self.nodecay_region()
        if hi > lo:
            self.grad[lo:hi].zero_()
        self.prezeroed = True

    # ------------------------------------------------------------------ regions
    def decay_region(self):
        return 0, self.n_decay

    def nodecay_region(self):
        return self.n_decay, self.numel

    def span(self, params: list[Param]) -> tuple[int, int]:
        """[lo, hi) of params that are laid out back-to-back (e.g. q/k/v kernels registered
        consecutively -> one fused [3*W, W] GEMM weight). Raises if they are not contiguous."""
        ps = sorted(params, key=lambda p: p.offset)
        for a, b in zip(ps, ps[1:]):
            if a.offset + a.numel != b.offset:
                raise ValueError(f"{a.name} and {b.name} are not contiguous in the arena")
        return ps[0].offset, ps[-1].offset + ps[-1].numel

    def num_parameters(self) -> int:
        return sum(p.numel for p in self.params)

    def by_name(self) -> dict[str, Param]:
        return {p.name: p for p in self.params}


def _init_values(spec: ParamSpec, gen: torch.Generator) -> torch.Tensor:
    t = _init_raw(spec, gen)
    return spec.post_init(t) if spec.post_init is not None else t


def _init_raw(spec: ParamSpec, gen: torch.Generator) -> torch.Tensor:
    shape = spec.shape
    if spec.init == "zeros":
        return torch.zeros(shape)
    if spec.init == "ones":
        return torch.ones(shape)
    if spec.init == "normal":
        return torch.randn(shape, generator=gen) * spec.std
    if spec.init == "trunc_normal":  # TF truncated_normal_initializer (BERT, Transformer)
        t = torch.empty(shape)
        torch.nn.init.trunc_normal_(t, 0.0, spec.std, -2 * spec.std, 2 * spec.std, generator=gen)
        return t
    if spec.init == "he_normal":
        return torch.randn(shape, generator=gen) * math.sqrt(2.0 / max(spec.fan_in, 1))
    if spec.init == "xavier_uniform":
        a = math.sqrt(6.0 / max(spec.fan_in + spec.fan_out, 1))
        return (torch.rand(shape, generator=gen) * 2 - 1) * a
    if spec.init == "uniform":
        a = 1.0 / math.sqrt(max(spec.fan_in, 1))
        return (torch.rand(shape, generator=gen) * 2 - 1) * a
    raise ValueError(f"unknown init {spec.init}")
