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
            alt = os.environ.get("TFK_C_PATH")
            if alt:
                # compile-time A/B: a second build of the extension (tools/build_variant.sh) loaded
                # under the same module name
                import importlib.util
                import sys
                spec = importlib.util.spec_from_file_location("tensorflow_k8s_amd._C", alt)
                C = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(C)
                sys.modules["tensorflow_k8s_amd._C"] = C
            else:
                from .. import _C as C  # noqa: N811
        except ImportError as e:  # pragma: no cover - exercised on misconfigured boxes only
            raise RuntimeError(
                "tfk native extension tensorflow_k8s_amd/_C is not built; run `python tools/build_ext.py` "
                f"(import error: {e})") from e
        _C = _OpProfiler(C) if os.environ.get("TFK_OPPROF") else C
    return _C


class _OpProfiler:
    """TFK_OPPROF=1: wraps every native entry point with a pair of device events on the current
    stream and records (name, compact args, elapsed ms) per call; ``records()`` synchronizes and
    resolves them. Used by tools/op_profile.py for per-layer kernel times; off in normal runs."""

    def __init__(self, mod):
        self._mod = mod
        self._pending = []
        self.__file__ = getattr(mod, "__file__", "")

    @staticmethod
    def _desc(a):
        if isinstance(a, torch.Tensor):
            return {"shape": list(a.shape), "esize": a.element_size()}
        if isinstance(a, (int, float, str, bool)) or a is None:
            return a
        if isinstance(a, (list, tuple)):
            return [_OpProfiler._desc(x) for x in a]
        return type(a).__name__

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn

        def wrapped(*args, **kw):
            if not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing():
                return fn(*args, **kw)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*args, **kw)
            e1.record()
            self._pending.append((name, [self._desc(a) for a in args], e0, e1))
            return r
        return wrapped

    def records(self, clear: bool = True):
        torch.cuda.synchronize()
        out = [{"op": n, "args": a, "ms": e0.elapsed_time(e1)} for n, a, e0, e1 in self._pending]
        if clear:
            self._pending = []
        return out


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
# split-K slab workspace slot of conv weight gradients; runtime/streams.py sets one per side stream
WGRAD_SLOT = "splitk_wgrad"
# True while runtime/streams.py issues weight gradients on a side stream (ops.gemm.conv_wgrad then
# sizes its split-K grid for running beside the critical path: SIDE_WGRAD_FILL_DIV)
ON_SIDE_STREAM = False


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
