#!/usr/bin/env python3
"""A/B of the g4 engine's tiles on model shapes, interleaved in one process (rules 24/25 of
cdna_hip_programming.md §5.4: random operands, rounds alternate the variants):
256x256 (16 waves, 2 stages), 128x128 (4 waves, 2 blocks/CU, 2 stages) and the 8-wave
one-block-per-CU 256x128 / 128x256 tiles with the 3-stage LDS ring, vs torch.matmul (hipBLASLt).

    python tools/tile_ab.py [--iters 20] [--rounds 3] [--only NAME] [--dirs fwd,dgrad,wgrad,conv]
One JSON line per (shape, direction): TFLOP/s median over rounds per tile.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def _engine(t, on: bool):
    """Switch the 256x256 engine a named tile stands for: "g8" (8-phase) or "g5" (mid-tile barrier)."""
    if t == "g8":
        lib().g8_set(1 if on else 0)
    elif t == "g5":
        lib().g5_set(8 if on else 0)
    elif t == "g5s":  # g5 with the fixed-slot schedule
        lib().g5_set(9 if on else 0)
    elif t == "g5t":  # fixed slots, DMA pieces late, MFMAs first in each slot
        lib().g5_set(10 if on else 0)


def _g8(fn, t):
    """Run fn on tile t; "g8" / "g5" = the 256x256 tile on that engine."""
    if not isinstance(t, str):
        return fn(t)
    _engine(t, True)
    try:
        return fn((256, 256))
    finally:
        _engine(t, False)


def tname(t):
    return t if isinstance(t, str) else f"t{t[0]}x{t[1]}"

DENSE = {  # name: (M, N, K)
    "sq4096": (4096, 4096, 4096),
    "bert_qkv": (8192, 2304, 768),
    "bert_ffn1": (8192, 3072, 768),
    "bert_ffn2": (8192, 768, 3072),
    "tfm_ffn1": (16384, 4096, 1024),
    "tfm_ffn2": (16384, 1024, 4096),
    "tfm_logits": (8192, 33728, 1024),
    "r50_s4_1x1": (50176, 1024, 256),
    "r50_s5_1x1": (12544, 2048, 512),
}
CONV = {  # ResNet-50 bs256 3x3 convs (N, H, W, C, K): stride 1
    "r50_3x3_s3": (256, 28, 28, 128, 128),
    "r50_3x3_s4": (256, 14, 14, 256, 256),
    "r50_3x3_s5": (256, 7, 7, 512, 512),
}
TILES = [(256, 256), (128, 128), (256, 128), (128, 256), "g8", "g5"]  # "g8"/"g5": 256x256 on that engine


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--dirs", default="fwd,dgrad,wgrad,conv")
    ap.add_argument("--tiles", default="", help="subset, e.g. 256x256,g8,g5")
    args = ap.parse_args()
    if args.tiles:
        TILES[:] = [t if t in ("g8", "g5", "g5s", "g5t") else tuple(int(v) for v in t.split("x")) for t in args.tiles.split(",")]
    dirs = set(args.dirs.split(","))
    dev = "cuda"
    for name, (M, N, K) in DENSE.items():
        if args.only and args.only not in name:
            continue
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        gw = torch.empty(N, K, device=dev, dtype=torch.float32)
        fl = 2.0 * M * N * K
        runs = {}
        if "fwd" in dirs:
            runs["fwd"] = ({t: (lambda t=t: _g8(lambda tt: G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN,
                                                                   G.EPI_BF16, tt), t)) for t in TILES}, lambda: x @ w.t())
        if "dgrad" in dirs:
            runs["dgrad"] = ({t: (lambda t=t: _g8(lambda tt: G._gemm(dy, w, dx, M, K, N, N, K, K, G.A_KIN, G.B_KOUT,
                                                                     G.EPI_BF16, tt), t)) for t in TILES}, lambda: dy @ w)
        if "wgrad" in dirs:
            runs["wgrad"] = ({t: (lambda t=t: _g8(lambda tt: G._gemm(dy, x, gw, N, K, M, N, K, K, G.A_KOUT, G.B_KOUT,
                                                                     G.EPI_F32, tt), t)) for t in TILES},
                             lambda: dy.t() @ x)
        ref = (x.float() @ w.float().t())
        for d, (fns, blas) in runs.items():
            res = {t: [] for t in TILES}
            res["blas"] = []
            for _ in range(args.rounds):
                for t, fn in fns.items():
                    res[t].append(fl / timeit(fn, args.iters) / 1e12)
                res["blas"].append(fl / timeit(blas, args.iters) / 1e12)
            out = {"shape": name, "dir": d, "M": M, "N": N, "K": K}
            for k, v in res.items():
                out["blas" if k == "blas" else tname(k)] = round(statistics.median(v), 1)
            if d == "fwd":  # correctness of every tile against fp32
                errs = {}
                for t, fn in fns.items():
                    fn()
                    errs[tname(t)] = round(float((y.float() - ref).norm() / ref.norm()), 5)
                out["rel_err"] = errs
            print(json.dumps(out), flush=True)
        del x, w, dy, y, dx, gw, ref
        torch.cuda.empty_cache()
    if "conv" not in dirs:
        return
    for name, (Nn, H, W, C, Kc) in CONV.items():
        TILES_C = list(TILES)
        if args.only and args.only not in name:
            continue
        g = G.ConvGeom(Nn, H, W, C, Kc, 3, 3, 1, 1, 1, 1)
        x = (torch.rand(Nn, H, W, C, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(Kc, 3, 3, C, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        fl = float(g.flops())
        res = {t: [] for t in TILES_C}
        outs = {}
        for _ in range(args.rounds):
            for t in TILES_C:
                G.FORCE_TILE = (256, 256) if isinstance(t, str) else t
                _engine(t, True)
                try:
                    res[t].append(fl / timeit(lambda: G.conv_fwd(x, w, g), args.iters) / 1e12)
                    outs[t] = G.conv_fwd(x, w, g)
                finally:
                    G.FORCE_TILE = None
                    _engine(t, False)
        ref = G._ref_conv(x, w, g)
        out = {"shape": name, "dir": "conv_fwd", "M": Nn * H * W, "N": Kc, "K": 9 * C}
        for t in TILES_C:
            out[tname(t)] = round(statistics.median(res[t]), 1)
        out["rel_err"] = {tname(t): round(float((outs[t].float() - ref).norm() / ref.norm()), 5) for t in TILES_C}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
