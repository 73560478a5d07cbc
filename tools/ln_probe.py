#!/usr/bin/env python3
"""LayerNorm backward (default: Transformer-big's 8192 x 1024 with the residual-branch gradient and
the consumer dropout fused, as the model runs it; --shape / --no-dres / --dbias for other call
forms, e.g. BERT-base: --shape 8192 768 --dbias): device-event time per call for rows-per-wave
settings (calls replayed from a captured graph), interleaved rounds in one process, outputs checked
against the default.
    python tools/ln_probe.py [--iters 50] [--rounds 5] [--shape M W] [--no-dres] [--dbias]"""
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
    ap.add_argument("--shape", type=int, nargs=2, default=(8192, 1024), metavar=("M", "W"))
    ap.add_argument("--no-dres", action="store_true", help="no residual-branch gradient")
    ap.add_argument("--dbias", action="store_true", help="also reduce the consumer's bias gradient")
    ap.add_argument("--no-drop", action="store_true", help="no fused consumer dropout")
    args = ap.parse_args()
    M, W = args.shape
    x = torch.randn(M, W, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, W, device="cuda").to(torch.bfloat16)
    gamma, beta = torch.rand(W, device="cuda") + 0.5, torch.zeros(W, device="cuda")
    _, mean, rstd = T.layernorm_fwd(x, gamma, beta)
    dg, db = torch.zeros(W, device="cuda"), torch.zeros(W, device="cuda")
    dres = None if args.no_dres else torch.randn(M, W, device="cuda").to(torch.bfloat16)  # residual branch
    dbias = torch.zeros(W, device="cuda") if args.dbias else None
    res, ref, err = {}, None, {}
    # (rows per wave, kernel: 0 = generic ln_bwd_kernel, 1 = width-specialized ln_bwd_fast_kernel)
    cfgs = ((8, 0), (8, 1), (4, 1), (2, 1))
    for _ in range(args.rounds):
        for rows, pf in cfgs:
            lib().ln_bwd_set_rows(rows)
            lib().ln_bwd_set_fast(pf)
            fn = lambda: T.layernorm_bwd(dy, x, gamma, mean, rstd, dg, db, dres=dres, drop=None if args.no_drop else (0.1, 5), dbias=dbias)  # noqa: E731
            out = fn()
            dxo = out[0] if isinstance(out, (tuple, list)) else out
            if ref is None:
                ref = dxo.float().clone()
            err[f"rows{rows}_fast{pf}"] = (dxo.float() - ref).abs().max().item()
            # the calls replay from one captured graph: host launch overhead (allocation, binding,
            # two launches per call) would otherwise set a ~20-25 us floor of its own
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(args.iters):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(f"rows{rows}_fast{pf}", []).append(e0.elapsed_time(e1) / args.iters * 1000.0)
    lib().ln_bwd_set_rows(8)
    lib().ln_bwd_set_fast(1)
    print(json.dumps({"shape": [M, W], "dres": dres is not None, "dbias": dbias is not None, "drop": not args.no_drop, "us_per_call": {k: round(statistics.median(v), 2) for k, v in res.items()},
                      "max_abs_dx_diff_vs_generic": err}))

if __name__ == "__main__":
    main()
