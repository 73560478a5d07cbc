#!/usr/bin/env python3
"""Cost of the BN-statistics epilogue (sharded f32 atomics) on ResNet-50's 1x1 conv forwards:
plain, 16 / 1 / 64 shards, device-event time per call (profiles/perf_log_r5.md: 64 shards on the
wide layers save ~20 us on the 64 -> 256 forward alone and nothing on the step).
    python tools/bn_stats_probe.py"""
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops import norm as BN
dev = "cuda"
def t(fn, it=30):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
for (H, C, K) in [(56, 64, 256), (56, 256, 64), (56, 64, 64), (28, 128, 512), (28, 512, 128)]:
    g = G.ConvGeom(256, H, H, C, K, 1, 1, 1, 1, 0, 0)
    x = torch.randn(256, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).to(torch.bfloat16)
    st = BN.BNState(K, dev, shards=16)
    a = t(lambda: G.conv_fwd(x, w, g))
    b = t(lambda: G.conv_fwd(x, w, g, st.stats, st.shards))
    st1 = BN.BNState(K, dev, shards=1)
    c = t(lambda: G.conv_fwd(x, w, g, st1.stats, 1))
    st64 = BN.BNState(K, dev, shards=64)
    d = t(lambda: G.conv_fwd(x, w, g, st64.stats, 64))
    M = 256 * H * H
    by = (M * C + M * K) * 2
    print(f"fwd 1x1 M{M} C{C}->K{K}: plain {a:.1f} us ({by/a/1e3:.0f} GB/s)  stats16 {b:.1f}  stats1 {c:.1f}  stats64 {d:.1f}", flush=True)
