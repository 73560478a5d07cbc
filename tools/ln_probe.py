#!/usr/bin/env python3
"""LayerNorm backward at Transformer-big's shape (8192 x 1024, bf16 mode with the consumer dropout
fused and the residual-stream gradient added, as the model runs it): device-event time per call for
(threads per block, rows per wave) settings of the grid, interleaved rounds in one process; the
outputs of every setting are checked against the (256, 8) one.
python tools/ln_probe.py [--iters 50] [--rounds 5]"""
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
    dres = torch.randn(M, W, device="cuda").to(torch.bfloat16)
    dg, db = torch.zeros(W, device="cuda"), torch.zeros(W, device="cuda")
    res, outs = {}, {}
    cfgs = [(256, 8), (512, 4), (512, 2), (256, 4)]
    for _ in range(args.rounds):
        for nt, rows in cfgs:
            lib().ln_bwd_set_nt(nt)
            lib().ln_bwd_set_rows(rows)
            fn = lambda: T.layernorm_bwd(dy, x, gamma, mean, rstd, dg, db, dres=dres, drop=(0.1, 5))  # noqa: E731
            dg.zero_(); db.zero_()
            o = fn()
            outs[(nt, rows)] = (o, dg.clone(), db.clone())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(f"nt{nt}_rows{rows}", []).append(e0.elapsed_time(e1) / args.iters * 1000.0)
    lib().ln_bwd_set_rows(8)
    lib().ln_bwd_set_nt(-1)

    def flat(o):
        return torch.cat([t.float().reshape(-1) for t in (o if isinstance(o, (tuple, list)) else [o])])
    ref = outs[cfgs[0]]
    err = {f"nt{k[0]}_rows{k[1]}": max(float((flat(v[i]) - flat(ref[i])).abs().max() / (flat(ref[i]).abs().max() + 1e-12))
                                      for i in range(3)) for k, v in outs.items()}
    print(json.dumps({"shape": [M, W], "us_per_call": {k: round(statistics.median(v), 2) for k, v in res.items()},
                      "max_rel_err_vs_nt256_rows8": err}))


if __name__ == "__main__":
    main()
