"""Measured GEMM configurations (autotuning table) for shapes whose best tile / split-K count the
analytic picker (ops.gemm.pick_tile) gets wrong.

The table is produced ON an MI355X by ``tools/wgrad_sweep.py --table`` (every tile x split-K
candidate timed including the split-K slab reduce, interleaved rounds, median) and shipped as
``tuned_wgrad.json`` next to this module; the runtime only reads it. Keys are the weight-gradient
GEMM shape gw[M][N] = dY[K][M]^T X[K][N] (M = output features, N = input features x taps,
K = pixels/tokens). A shape not in the table falls back to the analytic picker.
TFK_TUNING=0 disables the table (A/B).
"""
from __future__ import annotations

import json
import os

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_wgrad.json")
_TABLE: dict | None = None
ENABLED = os.environ.get("TFK_TUNING", "1") != "0"


def _load() -> dict:
    global _TABLE
    if _TABLE is None:
        _TABLE = {}
        try:
            with open(_PATH) as f:
                for e in json.load(f)["entries"]:
                    _TABLE[(int(e["M"]), int(e["N"]), int(e["K"]))] = (tuple(e["tile"]), int(e["splits"]))
        except (OSError, ValueError, KeyError):
            _TABLE = {}
    return _TABLE


def wgrad_config(M: int, N: int, K: int):
    """(tile, splits) measured best for this weight-gradient shape, or None."""
    if not ENABLED:
        return None
    return _load().get((M, N, K))
