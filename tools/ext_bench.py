#!/usr/bin/env python3
"""Cost of the GEMM epilogue extras on a Transformer-big FFN1 shape (M 8192, N 4096, K 1024):
plain / +relu / +aux / +dropout / all, for the bf16 g4 GEMM and the MX-fp8 GEMM (us per call)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import fp8 as F8  # noqa: E402
from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402


def us(f, iters=30):
    f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    for (M, N, K) in ((8192, 4096, 1024), (8192, 1024, 4096), (8192, 1024, 1024)):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16) * 0.05
        r = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        xq, wq = F8.mx_quantize(x), F8.mx_quantize(w)
        row = {"M": M, "N": N, "K": K}
        variants = {"plain": {}, "relu": {"act": 1}, "aux": {"aux": aux}, "drop": {"drop_p": 0.1},
                    "resid": {"resid": r}, "relu_aux_drop": {"act": 1, "aux": aux, "drop_p": 0.1},
                    "resid_drop": {"resid": r, "drop_p": 0.1}}
        for name, kw in variants.items():
            act = kw.get("act", 0)
            row[f"fp8_{name}"] = us(lambda: lib().gemm_mxfp8(xq[0], xq[1], wq[0], wq[1], y, M, N, K, None,
                                                                kw.get("resid"), act, kw.get("aux"),
                                                                kw.get("drop_p", 0.0), 7))
            row[f"bf16_{name}"] = us(lambda: G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16,
                                                     G.pick_tile(M, N, big_ok=True, K=K, g4=True), act=act,
                                                     resid=kw.get("resid"), aux=kw.get("aux"),
                                                     drop_p=kw.get("drop_p", 0.0), drop_seed=7))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
