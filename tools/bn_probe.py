#!/usr/bin/env python3
"""BatchNorm streaming passes at ResNet-50 bs256 shapes, each kernel alone on the GPU: device-event
time per call and effective HBM bandwidth of bn_apply (+relu +packed mask) and bn_bwd_apply (bitmask
relu), median of interleaved rounds. (Round 6 measured 5.0-6.8 TB/s, at the ~6.3 TB/s copy ceiling;
issuing 2 or 4 grid-stride iterations' loads up front measured slower: profiles/perf_log_r6.md.)
    python tools/bn_probe.py [--iters 20] [--rounds 3]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

# (rows = N*H*W, C): the stage shapes of ResNet-50 at batch 256
SHAPES = [(256 * 56 * 56, 64), (256 * 56 * 56, 256), (256 * 28 * 28, 512), (256 * 14 * 14, 1024), (256 * 7 * 7, 2048)]


def _time(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    out = {}
    for M, C in SHAPES:
        y = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        da = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        scale, shift = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
        coef = torch.randn(3 * C, device="cuda")
        a = torch.empty_like(y)
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda")
        dy = torch.empty_like(y)
        fwd = lambda: lib().bn_apply(y, scale, shift, None, None, None, True, a, M, C, mask)  # noqa: E731
        bwd = lambda: lib().bn_bwd_apply(da, mask, y, coef, dy, None, None, None, None, M, C, None, None)  # noqa: E731
        res = {}
        for _ in range(args.rounds):
            res.setdefault("fwd", []).append(_time(fwd, args.iters))
            res.setdefault("bwd", []).append(_time(bwd, args.iters))
        nb = M * C * 2
        bytes_ = {"fwd": 2 * nb + nb // 16, "bwd": 3 * nb + nb // 16}
        row = {}
        for k, v in res.items():
            us = statistics.median(v)
            row[k] = {"us": round(us, 2), "TB/s": round(bytes_[k] / us / 1e6, 2)}
        out[f"{M}x{C}"] = row
        print(json.dumps({f"{M}x{C}": row}), flush=True)
        del y, da, a, mask, dy
    print(json.dumps({"bn_probe": out}))


if __name__ == "__main__":
    main()
