#!/usr/bin/env python3
"""ResNet-50 (bs256) memory-bound pointwise GEMMs, each with and without its fused BN epilogue
work, timed with device events (interleaved rounds) -- and the driver for rocprofv3 PMC passes
on them (--reps N, no timing). Variants:
  fwd1x1        a2[M,64] @ w3 -> y3[M,256]            (+stats: BN batch statistics in the epilogue)
  dgrad1x1      dy[M,64] @ w1 -> dx[M,256]            (+bnr: mask, residual, BN-backward sums, dz store)
  conv3x3_s3    28x28x128 -> 128 3x3 forward          (+stats)

    python tools/pw_probe.py [--iters 20] [--rounds 3]      -> JSON lines
    rocprofv3 --pmc ... -- python3 tools/pw_probe.py --reps 5
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops import norm as BN  # noqa: E402


def r(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def variants():
    g = G.ConvGeom(256, 56, 56, 64, 256, 1, 1)
    x, w = r(256, 56, 56, 64), r(256, 1, 1, 64) * 0.1
    st = BN.BNState(256, "cuda")
    gd = G.ConvGeom(256, 56, 56, 256, 64, 1, 1)
    dy, w1 = r(256, 56, 56, 64), r(64, 1, 1, 256) * 0.1
    y3, res = r(256, 56, 56, 256), r(256, 56, 56, 256)
    st3 = BN.BNState(256, "cuda")
    mk = BN.pack_relu_mask(r(256, 56, 56, 256))
    g3 = G.ConvGeom(256, 28, 28, 128, 128, 3, 3, 1, 1, 1, 1)
    x3, w3 = r(256, 28, 28, 128), r(128, 3, 3, 128) * 0.05
    st33 = BN.BNState(128, "cuda")
    M = 256 * 56 * 56
    return {
        "fwd1x1": (lambda: G.conv_fwd(x, w, g), (M * 64 + M * 256) * 2),
        "fwd1x1+stats": (lambda: G.conv_fwd(x, w, g, st.stats, st.shards), (M * 64 + M * 256) * 2),
        "dgrad1x1": (lambda: G.conv_dgrad(dy, w1, gd), (M * 64 + M * 256) * 2),
        "dgrad1x1+resid": (lambda: G.conv_dgrad(dy, w1, gd, resid=res), (M * 64 + 2 * M * 256) * 2),
        "dgrad1x1+bnr": (lambda: G.conv_dgrad(dy, w1, gd, resid=res, bnr=BN.BNReduce(y3, st3, a=mk, premask=True)),
                         (M * 64 + 3 * M * 256) * 2 + M * 256 // 8),
        "conv3x3_s3": (lambda: G.conv_fwd(x3, w3, g3), (200704 * 128 * 2) * 2),
        "conv3x3_s3+stats": (lambda: G.conv_fwd(x3, w3, g3, st33.stats, st33.shards), (200704 * 128 * 2) * 2),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=0, help="profiler driver mode: run each variant N times, no timing")
    args = ap.parse_args()
    vs = variants()
    if args.reps:
        for _ in range(args.reps):
            for fn, _ in vs.values():
                fn()
        torch.cuda.synchronize()
        print("pw_probe done")
        return
    res = {k: [] for k in vs}
    for _ in range(args.rounds):
        for k, (fn, _) in vs.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) / args.iters * 1000.0)
    for k, (fn, nbytes) in vs.items():
        us = statistics.median(res[k])
        print(json.dumps({"variant": k, "us": round(us, 1), "TB_s": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
