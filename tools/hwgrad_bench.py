#!/usr/bin/env python3
"""Micro-benchmark of the halo-tile 3x3 weight gradient (csrc/kernels/conv_hwgrad.hip, incl. its
slab reduce) vs the im2col gather on the g4 engine, on every ResNet-50 bs256 3x3 conv shape.
One JSON line per (shape, path)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
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
    N = int(os.environ.get("N", 256))
    # (H, C, stride): ResNet-50 3x3 convs (stride-2 ones are the first block of stages 3-5)
    for (H, C, st) in [(56, 64, 1), (28, 128, 1), (14, 256, 1), (7, 512, 1), (56, 128, 2), (28, 256, 2),
                       (14, 512, 2)]:
        g = G.ConvGeom(N, H, H, C, C, 3, 3, st, st, 1, 1)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        dy = torch.randn(N, g.P, g.Q, C, device=dev).to(torch.bfloat16)
        gw = torch.zeros(C, 3, 3, C, device=dev)
        fl = 2.0 * N * g.P * g.Q * C * C * 9
        for hw in (True, False):
            G.HWGRAD = hw
            t = timeit(lambda: G.conv_wgrad(dy, x, g, gw))
            print(json.dumps({"shape": f"{H}x{H}x{C}/s{st}", "path": "halo" if hw else "gather",
                              "slabs": G.hwgrad_slabs(g) if hw else None, "ms": round(t, 4),
                              "TF/s": round(fl / t / 1e9, 1)}), flush=True)
        G.HWGRAD = True
    # ResNet conv1 (7x7/s2, 3 real of 8 channels): direct stem kernel vs the gather
    g = G.ConvGeom(N, 224, 224, 8, 64, 7, 7, 2, 2, 3, 3)
    x = torch.zeros(N, 224, 224, 8, device=dev, dtype=torch.bfloat16)
    x[..., :3] = torch.randn(N, 224, 224, 3, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, 112, 112, 64, device=dev).to(torch.bfloat16)
    gw = torch.zeros(64, 7, 7, 8, device=dev)
    fl = 2.0 * N * 112 * 112 * 64 * 49 * 3
    for cu in (3, None):
        t = timeit(lambda: G.conv_wgrad(dy, x, g, gw, cin_used=cu))
        print(json.dumps({"shape": "stem 224x224x3->64 7x7/s2", "path": "stem" if cu else "gather", "ms": round(t, 4),
                          "TF/s(real ch)": round(fl / t / 1e9, 1)}), flush=True)

    w = (torch.randn(64, 7, 7, 8, device=dev) * 0.1).to(torch.bfloat16)
    st = torch.zeros(16 * 2 * 64, device=dev)
    fl = 2.0 * N * 112 * 112 * 64 * 49 * 3
    for cu in (3, None):
        t = timeit(lambda: G.conv_fwd(x, w, g, stats=st, shards=16, cin_used=cu))
        print(json.dumps({"shape": "stem fwd 224x224x3->64 7x7/s2", "path": "stem" if cu else "gather",
                          "ms": round(t, 4), "TF/s(real ch)": round(fl / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
