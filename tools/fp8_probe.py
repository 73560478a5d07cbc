#!/usr/bin/env python3
"""Driver for rocprofv3 passes on one MX-fp8 GEMM shape vs the bf16 g4 GEMM of the same shape
(default: Transformer-big's 1024-wide projections, 8192 x 1024 x 1024, plain epilogue, both on
128x128 tiles), --reps dispatches each, no timing.

    rocprofv3 --pmc <counters> -- python3 tools/fp8_probe.py [--M 8192 --N 1024 --K 1024] [--reps 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import fp8 as F8  # noqa: E402
from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    M, N, K = a.M, a.N, a.K
    x = (torch.randn(M, K, device="cuda")).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    xq, xs = F8.mx_quantize(x)
    wq, ws = F8.mx_quantize(w)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(a.reps):
        lib().gemm_mxfp8(xq, xs, wq, ws, y, M, N, K, None, None, 0, None, 0.0, 0)
    for _ in range(a.reps):
        G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, (128, 128))
    torch.cuda.synchronize()
    print("fp8_probe done")


if __name__ == "__main__":
    main()
