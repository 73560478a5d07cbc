"""Fused softmax cross-entropy forward+backward (csrc/kernels/loss.hip)."""
from __future__ import annotations

import torch

from ._lib import lib, on_gpu


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, smoothing: float = 0.0, ignore_index: int = -100,
                 scale: float = 1.0, want_grad: bool = True, want_correct: bool = False, V: int | None = None):
    """Returns (per-row loss f32 [B], dlogits bf16 [B,ld] = scale*(softmax - target) or None, correct f32 [B] or None).
    V < logits.shape[1]: only the first V columns are classes (vocab padded to a multiple of 128);
    the padding columns of dlogits are zero."""
    B, ld = logits.shape
    V = ld if V is None else V
    if not on_gpu(logits):
        if V < ld:
            loss, d, corr = softmax_xent(logits[:, :V], labels, smoothing, ignore_index, scale, want_grad, want_correct)
            if d is not None:
                dp = torch.zeros(B, ld, dtype=torch.bfloat16)
                dp[:, :V] = d
                d = dp
            return loss, d, corr
        x = logits.float()
        lse = torch.logsumexp(x, dim=1)
        valid = (labels != ignore_index) & (labels >= 0) & (labels < V)
        lab = labels.clamp(0, V - 1).long()
        nll = lse - x.gather(1, lab[:, None])[:, 0]
        smooth = lse - x.mean(1)
        loss = torch.where(valid, (1 - smoothing) * nll + smoothing * smooth, torch.zeros_like(lse))
        d = None
        if want_grad:
            p = torch.softmax(x, dim=1)
            t = torch.full_like(p, smoothing / V)
            t.scatter_add_(1, lab[:, None], torch.full((B, 1), 1 - smoothing))
            d = (scale * (p - t) * valid[:, None]).to(torch.bfloat16)
        corr = ((x.argmax(1) == lab) & valid).float() if want_correct else None
        return loss, d, corr
    loss = torch.empty(B, dtype=torch.float32, device=logits.device)
    # the register kernel writes the padding columns itself; only the streaming kernel needs a zeroed buffer
    full = V == ld or bool(lib().xent_full_row(V, ld))
    d = (torch.empty_like(logits) if full else torch.zeros_like(logits)) if want_grad else None
    corr = torch.empty(B, dtype=torch.float32, device=logits.device) if want_correct else None
    lib().softmax_xent(logits, labels, B, V, ld, smoothing, ignore_index, scale, loss, d, corr)
    return loss, d, corr
