#!/usr/bin/env python3
"""GEMM micro-benchmark: tfk MFMA kernels (ops.gemm) vs torch.matmul (hipBLASLt) on the shapes the
models run (BERT-base / Transformer-big projections, ResNet-50 1x1 convs) + a square reference.

    python tools/gemm_bench.py [--iters 50] [--only NAME]
Prints one JSON line per shape: tfk and hipBLASLt TFLOP/s for fwd (NT), dgrad (NN) and wgrad (TN).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402

SHAPES = {  # name: (M, N, K)
    "sq4096": (4096, 4096, 4096),
    "bert_qkv": (8192, 2304, 768),
    "bert_ffn1": (8192, 3072, 768),
    "bert_ffn2": (8192, 768, 3072),
    "bert_ao": (8192, 768, 768),
    "tfm_ffn1": (16384, 4096, 1024),
    "tfm_ffn2": (16384, 1024, 4096),
    "tfm_logits": (8192, 33728, 1024),
    "r50_s1_1x1": (802816, 256, 64),
    "r50_s3_1x1": (50176, 1024, 256),
}


def timeit(fn, iters):
    for _ in range(3):
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
    ap.add_argument("--only", default="")
    ap.add_argument("--fp8", type=int, default=1, help="also time the MX-fp8 forward GEMM")
    args = ap.parse_args()
    dev = "cuda"
    for name, (M, N, K) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16) * 0.05
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        gw = torch.empty(N, K, device=dev, dtype=torch.float32)
        fl = 2.0 * M * N * K
        r = {"shape": name, "M": M, "N": N, "K": K}
        r["tfk_fwd"] = fl / timeit(lambda: G.linear_fwd(x, w), args.iters) / 1e12
        r["tfk_dgrad"] = fl / timeit(lambda: G.linear_dgrad(dy, w), args.iters) / 1e12
        r["tfk_wgrad"] = fl / timeit(lambda: G.linear_wgrad(dy, x, gw), args.iters) / 1e12
        if args.fp8 and K % 128 == 0:
            from tensorflow_k8s_amd.ops import fp8 as F8
            xq, wq = F8.mx_quantize(x), F8.mx_quantize(w)
            y8 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            G.lib().gemm_mxfp8(xq[0], xq[1], wq[0], wq[1], y8, M, N, K, None, None, 0, None, 0.0, 0)
            gemm8 = lambda: G.lib().gemm_mxfp8(xq[0], xq[1], wq[0], wq[1], y8, M, N, K, None, None, 0, None, 0.0, 0)  # noqa: E731
            r["tfk_mxfp8_gemm"] = fl / timeit(gemm8, args.iters) / 1e12
            r["tfk_mxfp8_fwd_incl_quant"] = fl / timeit(lambda: F8.linear_fwd_mx(x, w, wq=wq), args.iters) / 1e12
        r["blas_fwd"] = fl / timeit(lambda: x @ w.t(), args.iters) / 1e12
        r["blas_dgrad"] = fl / timeit(lambda: dy @ w, args.iters) / 1e12
        r["blas_wgrad"] = fl / timeit(lambda: dy.t() @ x, args.iters) / 1e12
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del x, w, dy, gw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
