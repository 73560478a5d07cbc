#!/usr/bin/env python3
"""Race screen of the g8 (8-phase, ping-pong) GEMM engine: it accumulates every output in the same
K order as the g4 256x256 tile, so its result must be BIT-IDENTICAL to g4's on every run. Runs each
shape/direction --reps times (random operands, fresh each round) and counts runs that differ.

    python tools/g8_screen.py [--reps 20]        -> one JSON line per (shape, dir) + a summary line
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 2304, 768), (2999, 1000, 512), (16384, 1024, 4096), (512, 768, 3072)]


def run(fn, g8):
    lib().g8_set(1 if g8 else 0)
    try:
        return fn()
    finally:
        lib().g8_set(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    bad_total = 0
    for M, N, K in SHAPES:
        for d in ("fwd", "dgrad", "wgrad"):
            bad = 0
            for r in range(args.reps):
                g = torch.Generator(device="cuda").manual_seed(r)
                if d == "fwd":
                    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                    fn = lambda: (G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, (256, 256)), y.clone())[1]
                elif d == "dgrad":
                    dy = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    w = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    y = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
                    fn = lambda: (G._gemm(dy, w, y, M, K, N, N, K, K, G.A_KIN, G.B_KOUT, G.EPI_BF16, (256, 256)), y.clone())[1]
                else:  # weight gradient gw[N][K] = dy^T x over the M rows, 4 split-K f32 slabs
                    dy = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
                    ns = int(G.lib().gemm_splits(M, 4))
                    ws = torch.empty(ns * N * K, device="cuda", dtype=torch.float32)
                    fn = lambda: (G._gemm(dy, x, ws, N, K, M, N, K, K, G.A_KOUT, G.B_KOUT, G.EPI_F32, (256, 256),
                                          splits=4, split_stride=N * K), ws.clone())[1]
                ref = run(fn, False)
                out = run(fn, True)
                torch.cuda.synchronize()
                if not torch.equal(ref, out):
                    bad += 1
            bad_total += bad
            print(json.dumps({"M": M, "N": N, "K": K, "dir": d, "reps": args.reps, "mismatching_runs": bad}), flush=True)
    print(json.dumps({"summary": "g8 vs g4 bitwise", "mismatching_runs": bad_total}), flush=True)
    sys.exit(1 if bad_total else 0)


if __name__ == "__main__":
    main()
