"""Split-K slab reduce timing: two-pass kernel vs the S <= 8 direct kernel (csrc/kernels/misc.hip).

Times `splitk_reduce` per mode (ops splitk_set_direct: 0 two-pass, 1 direct 1 column per lane,
2 direct 2 columns) over the linear weight-gradient slab shapes (Transformer-big / BERT-base
wgrads, halved split counts on the side streams), and checks the outputs are bit-identical where
the two-pass kernel runs one group. Usage: python tools/splitk_probe.py [--iters 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

SHAPES = [(2, 4096 * 1024), (4, 4096 * 1024), (2, 3072 * 1024), (4, 1024 * 1024), (8, 1024 * 1024),
          (2, 1024 * 1024), (4, 768 * 3072), (8, 768 * 768), (3, 100003)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    L = lib()
    for S, n in SHAPES:
        stride = (n + 3) // 4 * 4
        slabs = torch.randn(S * stride, device="cuda")
        base = torch.randn(n, device="cuda")
        row = {"S": S, "n": n, "MB": round((S + 2) * n * 4 / 2**20, 1)}
        outs = {}
        for mode in (0, 1, 2, 0, 1, 2):
            L.splitk_set_direct(mode)
            out = base.clone()
            L.splitk_reduce(slabs, S, stride, n, out, None, True, 1.0)
            outs[mode] = out
            o2 = base.clone()
            for _ in range(5):
                L.splitk_reduce(slabs, S, stride, n, o2, None, False, 1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                L.splitk_reduce(slabs, S, stride, n, o2, None, True, 1.0)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            row[f"us_m{mode}"] = min(row.get(f"us_m{mode}", 1e9), round(us, 2))
        one_group = S <= 4 or (n + 255) // 256 >= 1024
        row["bit_equal"] = bool(torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])) if one_group else None
        row["max_diff"] = float((outs[0] - outs[2]).abs().max())
        row["TBps_m2"] = round(row["MB"] * 2**20 / (row["us_m2"] * 1e-6) / 1e12, 2)
        print(json.dumps(row), flush=True)
    L.splitk_set_direct(2)


if __name__ == "__main__":
    main()
