#!/usr/bin/env python3
"""A/B micro-benchmark of the dense GEMM engines on the model shapes: the LDS-DMA engine (gemm_g4.hip)
at its 256x256 and 128x128 tiles vs the register-staged engine (gemm.hip, TFK_GEMM_ENGINE=reg) at
its best tile vs torch.matmul (hipBLASLt), on uniform random operands, interleaved in one process
(cdna_hip_programming.md §5.4 rules 24/25). Weight gradients run without split-K here.

    python tools/engine_bench.py [--iters 30] [--rounds 3] [--only NAME]
One JSON line per shape and direction: TFLOP/s median over rounds.
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

SHAPES = {
    "sq4096": (4096, 4096, 4096),
    "sq8192": (8192, 8192, 8192),
    "tfm_ffn1": (16384, 4096, 1024),
    "tfm_ffn2": (16384, 1024, 4096),
    "tfm_logits": (8192, 33728, 1024),
    "bert_ffn1": (8192, 3072, 768),
    "bert_ffn2": (8192, 768, 3072),
}


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
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    L = lib()
    dev = "cuda"
    t = (256, 256)
    for name, (M, N, K) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(M, N, device=dev) * 2 - 1).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        gw = torch.empty(N, K, device=dev, dtype=torch.float32)
        fl = 2.0 * M * N * K
        def runs(t):
            return {
                "fwd": lambda: G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, t),
                "dgrad": lambda: G._gemm(dy, w, dx, M, K, N, N, K, K, G.A_KIN, G.B_KOUT, G.EPI_BF16, t),
                "wgrad": lambda: G._gemm(dy, x, gw, N, K, M, N, K, K, G.A_KOUT, G.B_KOUT, G.EPI_F32, t),
            }
        blas = {"fwd": lambda: x @ w.t(), "dgrad": lambda: dy @ w, "wgrad": lambda: dy.t() @ x}
        arms = {"g4_256": (1, (256, 256)), "g4_128": (1, (128, 128)), "reg_256": (0, (256, 256)),
                "reg_128": (0, (128, 128))}
        res = {}
        for _ in range(args.rounds):
            for d in ("fwd", "dgrad", "wgrad"):
                for arm, (eng, t) in arms.items():
                    L.gemm_set_engine(eng)
                    res.setdefault(f"{arm}_{d}", []).append(fl / timeit(runs(t)[d], args.iters) / 1e12)
                res.setdefault(f"blas_{d}", []).append(fl / timeit(blas[d], args.iters) / 1e12)
        L.gemm_set_engine(1)
        out = {"shape": name, "M": M, "N": N, "K": K}
        out.update({k: round(statistics.median(v), 1) for k, v in res.items()})
        print(json.dumps(out), flush=True)
        del x, w, dy, y, dx, gw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
