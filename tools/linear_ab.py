#!/usr/bin/env python3
"""Tile A/B of the Transformer-big linear GEMMs through the production entry points (ops.gemm
linear_fwd / linear_dgrad, with the epilogue extras the model uses: relu + aux store + dropout on
FFN1, relu-backward on FFN2's dgrad, residual adds): pick_tile's choice vs forced 256x256 / 128x128,
device-event timing, interleaved rounds in one process.

    python tools/linear_ab.py [--iters 20] [--rounds 3]   -> one JSON line per (op, shape)
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402

M = 8192  # Transformer-big bs32 x 256 tokens
FWD = {  # name: (N, K, extras)
    "ffn1": (4096, 1024, "relu_aux_drop"),
    "ffn2": (1024, 4096, "resid"),
    "qkv": (3072, 1024, ""),
    "kv": (2048, 1024, ""),
    "o": (1024, 1024, "resid"),
    "logits": (33728, 1024, ""),
}
DGRAD = {  # name: (K_in = output cols of dx, N_out = reduction, extras)
    "ffn2": (4096, 1024, "dact_relu"),
    "ffn1": (1024, 4096, ""),
    "qkv": (1024, 3072, ""),
    "kv": (1024, 2048, ""),
    "o": (1024, 1024, ""),
    "logits": (1024, 33728, ""),
}


def r(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    orig = G.pick_tile
    # "nosplit": the picker's tile with the few-tile dgrad split-K off (ops.gemm._dgrad_splitk)
    variants = {"pick": None, "nosplit": "nosplit", "t256": (256, 256), "t128": (128, 128), "t256x128": (256, 128)}

    def timed(fn, tile):
        G.pick_tile = orig if tile in (None, "nosplit") else (lambda *a, **k: tile)
        split_max = G.DGRAD_SPLITK_MAX_TILES
        if tile == "nosplit":
            G.DGRAD_SPLITK_MAX_TILES = 0
        try:
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / args.iters * 1000.0
        finally:
            G.pick_tile = orig
            G.DGRAD_SPLITK_MAX_TILES = split_max

    jobs = []
    blas = {}
    for name, (N, K, ex) in FWD.items():
        x, w = r(M, K), r(N, K) * 0.05
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if "aux" in ex else None
        res = r(M, N) if ex == "resid" else None
        kw = dict(act="relu" if "relu" in ex else None, aux=aux, resid=res, drop_p=0.1 if "drop" in ex else 0.0,
                  drop_seed=3)
        jobs.append((f"fwd_{name}", 2.0 * M * N * K, (lambda x=x, w=w, kw=kw: G.linear_fwd(x, w, **kw)),
                     orig(M, N, big_ok=True, K=K, g4=True)))
        if not ex:
            blas[f"fwd_{name}"] = lambda x=x, w=w: x @ w.t()
    for name, (Kin, Nout, ex) in DGRAD.items():
        dy, w = r(M, Nout), r(Nout, Kin) * 0.05
        src = r(M, Kin) if ex else None
        kw = dict(dact_src=src, dact="relu") if ex else {}
        jobs.append((f"dgrad_{name}", 2.0 * M * Nout * Kin, (lambda dy=dy, w=w, kw=kw: G.linear_dgrad(dy, w, **kw)),
                     orig(M, Kin, big_ok=True, K=Nout, g4=True)))
        if not ex:
            blas[f"dgrad_{name}"] = lambda dy=dy, w=w: dy @ w
    res = {j[0]: {v: [] for v in variants} for j in jobs}
    for _ in range(args.rounds):
        for name, fl, fn, _ in jobs:
            for v, tile in variants.items():
                res[name][v].append(timed(fn, tile))
            if name in blas:
                res[name].setdefault("blas", []).append(timed(blas[name], None))
    for name, fl, fn, picked in jobs:
        out = {"op": name, "M": M, "picked": list(picked) if picked else None}
        for v in list(variants) + (["blas"] if name in blas else []):
            us = statistics.median(res[name][v])
            out[v + "_us"] = round(us, 1)
            out[v + "_tfs"] = round(fl / us / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
