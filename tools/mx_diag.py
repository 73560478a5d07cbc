#!/usr/bin/env python3
"""Pattern diagnostics for the MX-fp8 GEMM (prints error structure for structured inputs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_k8s_amd.ops import fp8 as F8  # noqa: E402


def show(name, x, w):
    y = F8.linear_fwd_mx(x.cuda(), w.cuda()).float().cpu()
    ref = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    err = (y - ref).abs()
    print(name, "rel", float(err.norm() / (ref.norm() + 1e-9)), "exact frac", float((err == 0).float().mean()))
    print(" y[:3,:6]", y[:3, :6].tolist())
    print(" r[:3,:6]", ref[:3, :6].tolist())
    bad = (err != 0).nonzero()
    if len(bad):
        print(" first bad", bad[:8].tolist(), "rows bad", sorted(set(bad[:, 0].tolist()))[:20],
              "cols bad", sorted(set(bad[:, 1].tolist()))[:20])


def main():
    torch.manual_seed(0)
    M = N = K = 128
    one = torch.ones(M, K, dtype=torch.bfloat16)
    ri = torch.randint(-8, 9, (M, K)).to(torch.bfloat16)
    rw = torch.randint(-8, 9, (N, K)).to(torch.bfloat16)
    show("ones", one, one)
    show("x=rand w=1", ri, one)
    show("x=1 w=rand", one, rw)
    show("rand", ri, rw)
    xs = ri.clone()
    xs[:, :32] *= 16
    show("rand scaled", xs, rw)
    kk = torch.zeros(M, K, dtype=torch.bfloat16)
    kk[:, 40] = 1
    show("x=e40 w=rand", kk, rw)
    q, s = F8.mx_quantize(xs.cuda())
    print("scales row0", s[0].tolist(), "q row0[:8]", q[0, :8].tolist())
    K = 1024
    show("K1024 rand", torch.randint(-8, 9, (256, K)).to(torch.bfloat16), torch.randint(-8, 9, (256, K)).to(torch.bfloat16))


if __name__ == "__main__":
    main()
