"""Fused optimizer kernels over flat parameter arenas (csrc/kernels/optim.hip)."""
from __future__ import annotations

import torch

from ._lib import lib, on_gpu


def opt_hyper(step: torch.Tensor, lr_table: torch.Tensor, lr_offset: int, b1: float, b2: float,
              hp: torch.Tensor) -> None:
    """Device schedule step (hipGraph-safe): step += 1; hp = {lr_table[min(step-1+off, T-1)],
    1 - b1^step, 1 - b2^step}. The optimizer kernels read hp instead of host scalars."""
    if not on_gpu(hp):
        s = int(step[0]) + 1
        step[0] = s
        i = min(max(s - 1 + lr_offset, 0), lr_table.numel() - 1)
        hp[0] = lr_table[i]
        hp[1] = 1 - b1 ** s
        hp[2] = 1 - b2 ** s
        return
    lib().opt_hyper(step, lr_table, lr_offset, b1, b2, hp)


def _hp(hp, lr, bc1=None, bc2=None):
    """Host view of the (lr, bc1, bc2) a kernel would use (CPU reference path)."""
    if hp is None:
        return lr, bc1, bc2
    return float(hp[0]), float(hp[1]), float(hp[2])


def sgd_(w, wb, g, m, lr, momentum=0.9, wd=0.0, nesterov=False, grad_scale=1.0, grad_scale_dev=None, hp=None):
    if not on_gpu(w):
        lr = _hp(hp, lr)[0]
        gs = grad_scale * (float(grad_scale_dev[0]) if grad_scale_dev is not None else 1.0)
        d = g * gs + wd * w
        m.mul_(momentum).add_(d)
        w.sub_(lr * (d + momentum * m if nesterov else m))
        if wb is not None:
            wb.copy_(w)
        return
    lib().sgd(w, wb, g, m, lr, momentum, wd, nesterov, grad_scale, grad_scale_dev, hp)


def adamw_(w, wb, g, m, v, lr, b1, b2, eps, wd, step, grad_scale=1.0, grad_scale_dev=None, hp=None):
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    if not on_gpu(w):
        lr, bc1, bc2 = _hp(hp, lr, bc1, bc2)
        gs = grad_scale * (float(grad_scale_dev[0]) if grad_scale_dev is not None else 1.0)
        gr = g * gs
        m.mul_(b1).add_((1 - b1) * gr)
        v.mul_(b2).add_((1 - b2) * gr * gr)
        w.sub_(lr * ((m / bc1) / ((v / bc2).sqrt() + eps) + wd * w))
        if wb is not None:
            wb.copy_(w)
        return
    lib().adamw(w, wb, g, m, v, lr, b1, b2, eps, wd, bc1, bc2, grad_scale, grad_scale_dev, hp)


def lamb_(w, wb, g, m, v, u, chunks, seg_norms, lr, b1, b2, eps, wd, step, grad_scale=1.0, grad_scale_dev=None, hp=None):
    """chunks: (start int64[n], len int32[n], seg int32[n]) over the flat arena."""
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    cstart, clen, cseg = chunks
    if not on_gpu(w):
        lr, bc1, bc2 = _hp(hp, lr, bc1, bc2)
        gs = grad_scale * (float(grad_scale_dev[0]) if grad_scale_dev is not None else 1.0)
        gr = g * gs
        m.mul_(b1).add_((1 - b1) * gr)
        v.mul_(b2).add_((1 - b2) * gr * gr)
        u.copy_((m / bc1) / ((v / bc2).sqrt() + eps) + wd * w)
        seg_norms.zero_()
        for s0, ln, sg in zip(cstart.tolist(), clen.tolist(), cseg.tolist()):
            seg_norms[2 * sg] += (w[s0:s0 + ln] ** 2).sum()
            seg_norms[2 * sg + 1] += (u[s0:s0 + ln] ** 2).sum()
        for s0, ln, sg in zip(cstart.tolist(), clen.tolist(), cseg.tolist()):
            wn, un = seg_norms[2 * sg].sqrt(), seg_norms[2 * sg + 1].sqrt()
            r = (wn / un) if (wn > 0 and un > 0) else 1.0
            w[s0:s0 + ln] -= lr * r * u[s0:s0 + ln]
        if wb is not None:
            wb.copy_(w)
        return
    seg_norms.zero_()
    lib().lamb(w, wb, g, m, v, u, cstart, clen, cseg, seg_norms, lr, b1, b2, eps, wd, bc1, bc2, grad_scale,
               grad_scale_dev, hp)


def global_norm_clip_coef(g: torch.Tensor, max_norm: float, ss: torch.Tensor, coef: torch.Tensor,
                          norm: torch.Tensor | None = None) -> None:
    """coef[0] = min(1, max_norm / ||g||) computed on device (no host sync)."""
    if not on_gpu(g):
        n = g.float().norm()
        if norm is not None:
            norm[0] = n
        coef[0] = min(1.0, max_norm / (float(n) + 1e-6)) if max_norm > 0 else 1.0
        return
    ss.zero_()
    lib().sumsq(g, ss)
    lib().clip_coef(ss, max_norm, coef, norm)


def cast_f32_bf16(x: torch.Tensor, y: torch.Tensor) -> None:
    if not on_gpu(x):
        y.copy_(x)
        return
    lib().cast_f32_bf16(x, y)


def cast_bf16_f32(x: torch.Tensor, y: torch.Tensor) -> None:
    if not on_gpu(x):
        y.copy_(x)
        return
    lib().cast_bf16_f32(x, y)
