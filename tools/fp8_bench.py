#!/usr/bin/env python3
"""MX-fp8 GEMM engines vs the bf16 g4 GEMM on the transformer shapes (TFLOP/s, GEMM only, operands
pre-quantized; plus the forward incl. the activation quantize pass).

    python tools/fp8_bench.py [--iters 20] [--only NAME]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import fp8 as F8  # noqa: E402
from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

SHAPES = {"tfm_ffn1": (16384, 4096, 1024), "tfm_ffn2": (16384, 1024, 4096), "tfm_qkv": (16384, 3072, 1024),
          "tfm_logits": (8192, 33728, 1024), "bert_ffn1": (8192, 3072, 768), "sq8192": (8192, 8192, 8192),
          # Transformer-big bs32 x 256 tokens: the shapes the benchmark step runs
          "tb_o": (8192, 1024, 1024), "tb_kv": (8192, 2048, 1024), "tb_qkv": (8192, 3072, 1024),
          "tb_ffn1": (8192, 4096, 1024), "tb_ffn2": (8192, 1024, 4096)}


def tflops(f, fl, iters):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        f()
    torch.cuda.synchronize()
    return round(fl / ((time.perf_counter() - t0) / iters) / 1e12, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    for name, (M, N, K) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        xq, wq = F8.mx_quantize(x), F8.mx_quantize(w)
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        fl = 2.0 * M * N * K
        row = {"shape": name, "M": M, "N": N, "K": K}
        gemm8 = lambda: lib().gemm_mxfp8(xq[0], xq[1], wq[0], wq[1], y, M, N, K, None, None, 0, None, 0.0, 0)  # noqa: E731
        ref = None
        for label, eng, tile in (("fp8_reg", 0, -1), ("fp8_g4_128", 1, 128), ("fp8_g4_256", 1, 256), ("fp8_g4_auto", 1, 0)):
            lib().fp8_set_engine(eng)
            lib().fp8_set_tile(tile)
            gemm8()
            torch.cuda.synchronize()
            if ref is None:
                ref = y.float().clone()
            else:
                err = float((y.float() - ref).abs().max() / (ref.abs().max() + 1e-9))
                if err > 1e-3:
                    row[label + "_mismatch"] = err
            row[label] = tflops(gemm8, fl, args.iters)
            if label == "fp8_g4_auto":
                row["fp8_fwd_incl_quant"] = tflops(lambda: F8.linear_fwd_mx(x, w, wq=wq), fl, args.iters)
        lib().fp8_set_engine(-1)
        lib().fp8_set_tile(-1)
        row["bf16_g4"] = tflops(lambda: G.linear_fwd(x, w, out=y), fl, args.iters)
        row["bf16_blas"] = tflops(lambda: x @ w.t(), fl, args.iters)
        # backward GEMMs through the production entry points (fp8: incl. their quantize passes)
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        gw = torch.zeros(N, K, device="cuda")
        if N % 128 == 0:
            row["fp8_dgrad_incl_quant"] = tflops(lambda: F8.linear_dgrad_mx(dy, w), fl, args.iters)
        row["bf16_dgrad"] = tflops(lambda: G.linear_dgrad(dy, w), fl, args.iters)
        if M % 128 == 0:
            row["fp8_wgrad_incl_quant"] = tflops(lambda: F8.linear_wgrad_mx(dy, x, gw), fl, args.iters)
        row["bf16_wgrad"] = tflops(lambda: G.linear_wgrad(dy, x, gw), fl, args.iters)
        del dy, gw
        print(json.dumps(row), flush=True)
        del x, w, xq, wq, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
