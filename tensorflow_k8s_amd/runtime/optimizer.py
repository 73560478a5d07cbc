"""Optimizers over a ParamArena: one fused launch per parameter group (decay / no-decay).

Slot names follow TF (`Momentum`, `Adam`, `Adam_1`) so checkpoints carry optimizer state the way
TF-era TFJob workloads did.
"""
from __future__ import annotations

import math

import torch

from ..ops import optim as O
from .arena import ParamArena


class LRSchedule:
    """Linear warmup then cosine/poly/constant decay (per step)."""

    def __init__(self, base_lr: float, warmup: int = 0, total: int = 0, kind: str = "constant", end_lr: float = 0.0,
                 power: float = 1.0):
        self.base, self.warmup, self.total, self.kind, self.end, self.power = base_lr, warmup, total, kind, end_lr, power

    def __call__(self, step: int) -> float:
        if self.warmup and step < self.warmup:
            return self.base * (step + 1) / self.warmup
        if self.kind == "constant" or self.total <= self.warmup:
            return self.base
        t = min(1.0, (step - self.warmup) / max(1, self.total - self.warmup))
        if self.kind == "cosine":
            return self.end + (self.base - self.end) * 0.5 * (1 + math.cos(math.pi * t))
        if self.kind == "poly":
            return self.end + (self.base - self.end) * (1 - t) ** self.power
        return self.base


class Optimizer:
    slot_names: tuple = ()

    def __init__(self, arena: ParamArena, lr, weight_decay: float = 0.0):
        self.arena = arena
        self.lr = lr if callable(lr) else LRSchedule(lr)
        self.wd = weight_decay
        self.step_count = 0
        self.grad_scale = 1.0          # e.g. 1/world for gradient averaging
        self.grad_scale_dev = None     # device scalar (global-norm clipping)
        self.region = None             # (start, end) restrict to a shard (parameter-server)
        self._dev = None               # device schedule state (hipGraph capture), see enable_device_schedule
        for s in self.slot_names:
            arena.slot(s)

    # Adam-family bias-correction bases (SGD has none)
    _betas = (0.0, 0.0)

    def enable_device_schedule(self, max_steps: int = 200_000) -> None:
        """Move the per-step host scalars -- learning rate, step counter and Adam bias corrections --
        onto the device, so a hipGraph-captured step replays a correct update every time (a captured
        host scalar would freeze at its capture-time value). The LR schedule is tabulated on device
        for steps [0, T): T covers warmup + decay of an LRSchedule, else max_steps."""
        dev = self.arena.device
        if isinstance(self.lr, LRSchedule):
            T = max(1, (self.lr.total if self.lr.kind != "constant" else 0), self.lr.warmup) + 1
        else:
            T = max_steps
        table = torch.tensor([self.lr(i) for i in range(T)], dtype=torch.float32, device=dev)
        self._dev = {"step": torch.tensor([self.step_count], dtype=torch.int32, device=dev),
                     "lr": table, "hp": torch.zeros(3, dtype=torch.float32, device=dev)}

    def _device_hp(self):
        """Advance the device schedule (inside the step, hence inside a captured graph)."""
        if self._dev is None:
            return None
        if self._frozen:
            return self._dev["hp"]
        b1, b2 = self._betas
        O.opt_hyper(self._dev["step"], self._dev["lr"], 0, b1, b2, self._dev["hp"])
        return self._dev["hp"]

    _frozen = False

    def step_region(self, advance: bool = True) -> None:
        """Update ``self.region`` as one part of a global step that spans several region calls (the
        collective parameter server updates its shard bucket by bucket): the first call
        (advance=True) advances the step counter / device schedule, later calls of the same global
        step reuse its learning rate and bias corrections."""
        if advance:
            self._before = self.step_count
            self.step()
            return
        after = self.step_count
        self.step_count, self._frozen = self._before, True
        try:
            self.step()
        finally:
            self.step_count, self._frozen = after, False

    def sync_step(self) -> int:
        """Host step counter (reads the device counter when the schedule lives on device)."""
        if self._dev is not None:
            self.step_count = int(self._dev["step"][0].item())
        return self.step_count

    def _regions(self):
        lo, hi = self.region if self.region is not None else (0, self.arena.numel)
        d0, d1 = self.arena.decay_region()
        out = []
        a, b = max(lo, d0), min(hi, d1)
        if b > a:
            out.append((a, b, self.wd))
        n0, n1 = self.arena.nodecay_region()
        a, b = max(lo, n0), min(hi, n1)
        if b > a:
            out.append((a, b, 0.0))
        return out

    def state_dict(self):
        return {"step": self.sync_step()}

    def load_state_dict(self, d):
        self.step_count = int(d.get("step", 0))
        if self._dev is not None:
            self._dev["step"].fill_(self.step_count)


class SGD(Optimizer):
    slot_names = ("Momentum",)

    def __init__(self, arena, lr, momentum: float = 0.9, weight_decay: float = 5e-5, nesterov: bool = False):
        super().__init__(arena, lr, weight_decay)
        self.momentum, self.nesterov = momentum, nesterov

    def step(self):
        a = self.arena
        lr = self.lr(self.step_count)
        hp = self._device_hp()
        m = a.slot("Momentum")
        for lo, hi, wd in self._regions():
            O.sgd_(a.master[lo:hi], a.compute[lo:hi], a.grad[lo:hi], m[lo:hi], lr, self.momentum, wd, self.nesterov,
                   self.grad_scale, self.grad_scale_dev, hp=hp)
        self.step_count += 1


class AdamW(Optimizer):
    slot_names = ("Adam", "Adam_1")

    def __init__(self, arena, lr, b1=0.9, b2=0.999, eps=1e-6, weight_decay=0.01):
        super().__init__(arena, lr, weight_decay)
        self.b1, self.b2, self.eps = b1, b2, eps
        self._betas = (b1, b2)

    def step(self):
        a = self.arena
        self.step_count += 1
        lr = self.lr(self.step_count - 1)
        hp = self._device_hp()
        m, v = a.slot("Adam"), a.slot("Adam_1")
        for lo, hi, wd in self._regions():
            O.adamw_(a.master[lo:hi], a.compute[lo:hi], a.grad[lo:hi], m[lo:hi], v[lo:hi], lr, self.b1, self.b2,
                     self.eps, wd, self.step_count, self.grad_scale, self.grad_scale_dev, hp=hp)


class LAMB(Optimizer):
    """Layer-wise adaptive moments (BERT pretraining); trust ratio per parameter tensor."""
    slot_names = ("Adam", "Adam_1")
    CHUNK = 4096

    def __init__(self, arena, lr, b1=0.9, b2=0.999, eps=1e-6, weight_decay=0.01):
        super().__init__(arena, lr, weight_decay)
        self.b1, self.b2, self.eps = b1, b2, eps
        self._betas = (b1, b2)
        self._tables = {}
        self._u = torch.zeros(arena.numel, dtype=torch.float32, device=arena.device)
        self._norms = torch.zeros(2 * len(arena.params), dtype=torch.float32, device=arena.device)

    def _chunks(self, lo, hi):
        key = (lo, hi)
        if key not in self._tables:
            starts, lens, segs = [], [], []
            for p in self.arena.params:
                s, e = max(p.offset, lo), min(p.offset + p.numel, hi)
                for c in range(s, e, self.CHUNK):
                    starts.append(c - lo); lens.append(min(self.CHUNK, e - c)); segs.append(p.index)
            dev = self.arena.device
            self._tables[key] = (torch.tensor(starts, dtype=torch.int64, device=dev),
                                 torch.tensor(lens, dtype=torch.int32, device=dev),
                                 torch.tensor(segs, dtype=torch.int32, device=dev))
        return self._tables[key]

    def step(self):
        a = self.arena
        self.step_count += 1
        lr = self.lr(self.step_count - 1)
        hp = self._device_hp()
        m, v = a.slot("Adam"), a.slot("Adam_1")
        for lo, hi, wd in self._regions():
            O.lamb_(a.master[lo:hi], a.compute[lo:hi], a.grad[lo:hi], m[lo:hi], v[lo:hi], self._u[lo:hi],
                    self._chunks(lo, hi), self._norms, lr, self.b1, self.b2, self.eps, wd, self.step_count,
                    self.grad_scale, self.grad_scale_dev, hp=hp)
