"""Loader for the in-tree gfx950 kernel library (``tensorflow_k8s_amd/_C*.so``).

GPU tensors ALWAYS go through the HIP kernels; if the extension is missing on a GPU box this
raises instead of silently falling back to stock torch ops. CPU tensors use the fp32 torch
reference implementations in each ops module (used by the CPU test tier and as numerics oracle).
"""
from __future__ import annotations

import os

import torch

_C = None


def lib():
    global _C
    if _C is None:
        try:
            from .. import _C as C  # noqa: N811
        except ImportError as e:  # pragma: no cover - exercised on misconfigured boxes only
            raise RuntimeError(
                "tfk native extension tensorflow_k8s_amd/_C is not built; run `python tools/build_ext.py` "
                f"(import error: {e})") from e
        _C = C
    return _C


def available() -> bool:
    try:
        lib()
        return True
    except RuntimeError:
        return False


def on_gpu(*ts) -> bool:
    """True if the (first defined) tensor lives on the GPU -> HIP kernel path."""
    for t in ts:
        if t is not None:
            return t.is_cuda
    return False


# ---------------------------------------------------------------- workspaces
_ws: dict = {}


def workspace(device: torch.device, numel: int, dtype=torch.float32, slot: str = "splitk") -> torch.Tensor:
    """Grow-only scratch buffer per (device, slot). Stream-ordered reuse is safe because every
    consumer of a workspace runs on the same stream as its producer."""
    key = (str(device), slot, dtype)
    t = _ws.get(key)
    if t is None or t.numel() < numel:
        n = max(numel, int(t.numel() * 1.5) if t is not None else 0)
        t = torch.empty(n, dtype=dtype, device=device)
        _ws[key] = t
    return t[:numel]


def reset_workspaces() -> None:
    _ws.clear()


DEBUG = os.environ.get("TFK_DEBUG", "0") == "1"
