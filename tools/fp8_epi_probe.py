#!/usr/bin/env python3
"""Epilogue cost of the MX-fp8 GEMM on Transformer-big's FFN1 forward (8192 x 4096 x 1024): plain
bf16 output, EXT (relu + 1-bit mask aux + dropout), EXT_MX (+ both MX copies of the output) with and
without the bf16 store. --reps dispatches of each, for a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --stats -- python3 tools/fp8_epi_probe.py [--reps 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import fp8 as F8  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    M, N, K = 8192, 4096, 1024
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.zeros(N, device="cuda")
    xq, xs = F8.mx_quantize(x)
    wq, ws = F8.mx_quantize(w)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    m = torch.empty(M, N // 8, device="cuda", dtype=torch.uint8)
    mo = list(F8._mx_bufs(M, N, "cuda"))
    runs = {
        "plain": dict(),
        "ext": dict(act=1, aux=m, drop_p=0.1),
        "ext_mx": dict(act=1, aux=m, drop_p=0.1, mx_out=mo),
        "ext_mx_skip": dict(act=1, aux=m, drop_p=0.1, mx_out=mo, mx_skip_c=True),
    }
    for name, kw in runs.items():
        for _ in range(a.reps):
            lib().gemm_mxfp8(xq, xs, wq, ws, y, M, N, K, b, None, kw.get("act", 0), kw.get("aux"),
                             kw.get("drop_p", 0.0), 3, mx_out=kw.get("mx_out"), mx_skip_c=kw.get("mx_skip_c", False))
        torch.cuda.synchronize()
        print(name, "done", flush=True)


if __name__ == "__main__":
    main()
