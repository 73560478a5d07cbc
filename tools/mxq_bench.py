#!/usr/bin/env python3
"""Micro-benchmark of the MX-fp8 quantizers (csrc/kernels/fp8.hip) on Transformer-big shapes:
effective HBM GB/s (bf16 read + e4m3/e8m0 writes) of the dual (row + column) quantizer, the row
quantizer and the transposing quantizer. One JSON line per (op, shape)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import fp8 as F8  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    for R, C in [(8192, 1024), (8192, 3072), (8192, 4096), (1024, 1024), (4096, 1024), (33792, 1024)]:
        x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
        n = R * C
        for op, fn, by in (("dual", lambda: F8.mx_quantize_dual(x), n * 2 + 2 * n + 2 * n // 32),
                           ("row", lambda: F8.mx_quantize(x), n * 2 + n + n // 32),
                           ("t", lambda: F8.mx_quantize_t(x), n * 2 + n + n // 32)):
            t = timeit(fn)
            print(json.dumps({"op": op, "shape": [R, C], "us": round(t * 1e3, 2), "GB/s": round(by / t / 1e6, 1)}),
                  flush=True)
    # every fp8 weight of Transformer-big (+ the tied 33792x1024 table): per-tensor launches vs ONE
    # grouped launch (GroupQuantizer)
    W, F = 1024, 4096
    shapes = ([(3 * W, W), (W, W), (F, W), (W, F)] * 6 + [(3 * W, W), (W, W), (W, W), (2 * W, W), (W, W), (F, W), (W, F)] * 6
              + [(33792, W)])
    ws = [torch.randn(*sh, device="cuda").to(torch.bfloat16) for sh in shapes]
    by = sum(w.numel() * 4 + 2 * w.numel() // 32 for w in ws)
    gq = F8.GroupQuantizer(ws)
    for op, fn in (("weights_per_tensor", lambda: [F8.mx_quantize_dual(w) for w in ws]), ("weights_group", gq.run)):
        t = timeit(fn, iters=20)
        print(json.dumps({"op": op, "tensors": len(ws), "us": round(t * 1e3, 2), "GB/s": round(by / t / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
