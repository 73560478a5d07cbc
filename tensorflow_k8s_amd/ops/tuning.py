"""Measured GEMM configurations (autotuning tables) for shapes whose best tile / split-K count the
analytic picker (ops.gemm.pick_tile) gets wrong.

* ``tuned_wgrad.json`` (tools/wgrad_sweep.py): weight-gradient GEMMs, tile + split-K;
* ``tuned_conv.json`` (tools/conv_sweep.py): the tile of every conv forward ("fwd"), pointwise
  dgrad ("dgrad_pw") and stride-1 dgrad-as-forward ("dgrad_fwd") GEMM, keyed by the conv geometry
  and timed with the model's own epilogue (BN statistics / fused BN-backward reduction).

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

# TFK_WGRAD_TABLE: an alternative weight-gradient table (A/B of a fresh tools/wgrad_sweep.py --table)
_PATH = os.environ.get("TFK_WGRAD_TABLE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                            "tuned_wgrad.json")
# TFK_CONV_TABLE: an alternative conv tile table (A/B of a fresh tools/conv_sweep.py --table)
_CONV_PATH = os.environ.get("TFK_CONV_TABLE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                "tuned_conv.json")
_TABLE: dict | None = None
_CONV: dict | None = None
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


def _load_conv() -> dict:
    global _CONV
    if _CONV is None:
        _CONV = {}
        try:
            with open(_CONV_PATH) as f:
                for e in json.load(f)["entries"]:
                    _CONV[(e["kind"], tuple(int(v) for v in e["geom"]))] = tuple(e["tile"])
        except (OSError, ValueError, KeyError):
            _CONV = {}
    return _CONV


def conv_tile(kind: str, geom: tuple):
    """Measured best tile of a conv GEMM (kind: fwd | dgrad_pw | dgrad_fwd), or None."""
    if not ENABLED:
        return None
    return _load_conv().get((kind, tuple(geom)))
