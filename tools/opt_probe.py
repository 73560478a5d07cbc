"""Fused AdamW update alone on the GPU: time per call and effective HBM bandwidth (30 B/param:
f32 w, g, m, v read; w, m, v written; bf16 weight copy written) at Transformer-big's parameter count.
Compile-time variants load through TFK_C_PATH (tools/build_variant.sh).
    python tools/opt_probe.py [--params 210000000] [--iters 10]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=210_000_000)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    n = args.params
    w, g, m, v = (torch.randn(n, device="cuda") * 0.01 for _ in range(4))
    v.abs_()
    wb = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    L = lib()
    ref = w.clone(), m.clone(), v.clone()
    L.adamw(w, wb, g, m, v, 1e-3, 0.9, 0.98, 1e-8, 0.01, 0.1, 0.02, 1.0, None, None)
    # reference of one update (same formula in f32)
    w0, m0, v0 = ref
    mm = 0.9 * m0 + 0.1 * g
    vv = 0.98 * v0 + 0.02 * g * g
    we = w0 - 1e-3 * ((mm / 0.1) / (torch.sqrt(vv / 0.02) + 1e-8) + 0.01 * w0)
    err = float((w - we).abs().max())
    for _ in range(3):
        L.adamw(w, wb, g, m, v, 1e-3, 0.9, 0.98, 1e-8, 0.01, 0.1, 0.02, 1.0, None, None)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        L.adamw(w, wb, g, m, v, 1e-3, 0.9, 0.98, 1e-8, 0.01, 0.1, 0.02, 1.0, None, None)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    print(json.dumps({"variant": os.environ.get("TFK_C_PATH", "default"), "params": n, "us": round(us, 1),
                      "TBps": round(30 * n / (us * 1e-6) / 1e12, 2), "max_abs_err_vs_torch": err}), flush=True)


if __name__ == "__main__":
    main()
