#!/usr/bin/env python3
"""Micro-benchmark of the halo-tile 3x3 conv (csrc/kernels/conv_halo.hip) vs the implicit-GEMM
gather on ResNet-50 bs256 shapes: forward with BN statistics, dgrad (as a forward conv over dY)
with the BN-backward reduce + premasked dz store. One JSON line per (shape, op, halo)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops import norm as BN  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def timeit(fn, iters=30):
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
    dev = "cuda"
    for (N, HW, C) in [(256, 56, 64), (256, 28, 128)]:
        g = G.ConvGeom(N, HW, HW, C, C, 3, 3, 1, 1, 1, 1)
        x = torch.randn(N, HW, HW, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.randn(N, HW, HW, C, device=dev).to(torch.bfloat16)
        st = BN.BNState(C, dev)
        stats = torch.zeros(16 * 2 * C, device=dev)
        fl = 2.0 * N * HW * HW * C * C * 9
        for halo in (1, 0):
            lib().halo_set(halo)
            t_f = timeit(lambda: G.conv_fwd(x, w, g, stats=stats, shards=16))
            t_d = timeit(lambda: G.conv_dgrad(x, w, g, bnr=BN.BNReduce(y, st, premask=True)))
            lib().halo_set(-1)
            for op, t in (("fwd+stats", t_f), ("dgrad+bnr", t_d)):
                print(json.dumps({"shape": f"{HW}x{HW}x{C}", "op": op, "halo": halo, "ms": round(t, 4),
                                  "TF/s": round(fl / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
