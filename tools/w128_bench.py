#!/usr/bin/env python3
"""A/B of the 256x256 GEMM engines on the model shapes: g4 (16 waves, 64x64 wave tiles) vs the w128
variants (4 waves, 128x128 wave tiles; csrc/kernels/gemm_w128.h) vs torch.matmul (hipBLASLt).

    python tools/w128_bench.py [--iters 20] [--rounds 3] [--only NAME] [--variants 0,1,2,3,4]

Each variant's output is checked against variant 0 (g4) first. Prints one JSON line per shape and
direction: TFLOP/s per variant (median over interleaved rounds) and blas.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402

SHAPES = {  # name: (M, N, K)
    "sq4096": (4096, 4096, 4096),
    "sq8192": (8192, 8192, 8192),
    "bert_qkv": (8192, 2304, 768),
    "bert_ffn1": (8192, 3072, 768),
    "bert_ffn2": (8192, 768, 3072),
    "tfm_ffn1": (16384, 4096, 1024),
    "tfm_ffn2": (16384, 1024, 4096),
    "tfm_qkv": (16384, 3072, 1024),
    "tfm_logits": (8192, 33728, 1024),
}


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="0,1,2,3,4")
    args = ap.parse_args()
    vs = [int(v) for v in args.variants.split(",")]
    lib = G.lib()
    dev = "cuda"
    T = (256, 256)
    for name, (M, N, K) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        g = torch.Generator(device=dev).manual_seed(1)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        dy = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        gw = torch.empty(N, K, device=dev, dtype=torch.float32)
        ops = {
            "fwd": (lambda: G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, T), y, lambda: x @ w.t()),
            "dgrad": (lambda: G._gemm(dy, w, dx, M, K, N, N, K, K, G.A_KIN, G.B_KOUT, G.EPI_BF16, T), dx, lambda: dy @ w),
            "wgrad": (lambda: G._gemm(dy, x, gw, N, K, M, N, K, K, G.A_KOUT, G.B_KOUT, G.EPI_F32, T), gw,
                      lambda: dy.t() @ x),
        }
        fl = 2.0 * M * N * K
        for d, (run, out, blas) in ops.items():
            ref = None
            res = {"shape": name, "dir": d, "M": M, "N": N, "K": K}
            bad = []
            for v in vs:
                lib.w128_set(v)
                out.zero_()
                run()
                torch.cuda.synchronize()
                o = out.float()
                if ref is None:
                    ref = o.clone()
                else:
                    err = float((o - ref).abs().max()) / (float(ref.abs().max()) + 1e-9)
                    if not err < 1e-2:
                        bad.append((v, err))
            res["mismatch"] = bad
            times = {v: [] for v in vs}
            tb = []
            for _ in range(args.rounds):
                for v in vs:
                    if any(b[0] == v for b in bad):
                        continue
                    lib.w128_set(v)
                    times[v].append(timed(run, args.iters))
                tb.append(timed(blas, args.iters))
            for v in vs:
                if times[v]:
                    res[f"v{v}"] = round(fl / statistics.median(times[v]) / 1e12, 1)
            res["blas"] = round(fl / statistics.median(tb) / 1e12, 1)
            print(json.dumps(res), flush=True)
        lib.w128_set(-1)
        del x, w, dy, y, dx, gw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
