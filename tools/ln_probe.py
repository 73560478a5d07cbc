#!/usr/bin/env python3
"""LayerNorm backward at Transformer-big's shape (8192 x 1024, bf16 mode with the consumer dropout
fused, as the model runs it): device-event time per call for rows-per-wave settings of the grid,
interleaved rounds in one process.   python tools/ln_probe.py [--iters 50] [--rounds 5]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import transformer as T  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    M, W = 8192, 1024
    x = torch.randn(M, W, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, W, device="cuda").to(torch.bfloat16)
    gamma, beta = torch.rand(W, device="cuda") + 0.5, torch.zeros(W, device="cuda")
    _, mean, rstd = T.layernorm_fwd(x, gamma, beta)
    dg, db = torch.zeros(W, device="cuda"), torch.zeros(W, device="cuda")
    res = {}
    for _ in range(args.rounds):
        for rows in (8, 4, 2, 1):
            lib().ln_bwd_set_rows(rows)
            fn = lambda: T.layernorm_bwd(dy, x, gamma, mean, rstd, dg, db, drop=(0.1, 5))  # noqa: E731
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(rows, []).append(e0.elapsed_time(e1) / args.iters * 1000.0)
    lib().ln_bwd_set_rows(8)
    print(json.dumps({"shape": [M, W], "us_per_call_by_rows_per_wave": {r: round(statistics.median(v), 2)
                                                                          for r, v in res.items()}}))


if __name__ == "__main__":
    main()
