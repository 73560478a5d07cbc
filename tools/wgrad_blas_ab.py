#!/usr/bin/env python3
"""Weight-gradient GEMMs gw[N][K] (f32) = dy[M][N]^T x[M][K]: the framework's path (ops.gemm.
linear_wgrad: g4 tiles + split-K slabs + splitk_reduce, tuned table) vs hipBLASLt through
aten::mm.dtype_out (bf16 in, f32 out, no slabs), on the Transformer-big and ResNet-50 1x1 shapes.
Device-event timing, interleaved rounds.   python tools/wgrad_blas_ab.py [--iters 20] [--rounds 3]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402

SHAPES = {  # name: (N, K, M) -- gw is N x K, reduction over M
    "tb_o": (1024, 1024, 8192), "tb_qkv": (3072, 1024, 8192), "tb_kv": (2048, 1024, 8192),
    "tb_ffn1": (4096, 1024, 8192), "tb_ffn2": (1024, 4096, 8192), "tb_emb": (33728, 1024, 8192),
    "r50_s1": (256, 64, 802816), "r50_s1b": (64, 256, 802816), "r50_s2": (512, 128, 200704),
    "r50_s3": (1024, 256, 50176), "r50_s4": (2048, 512, 12544),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    for name, (N, K, M) in SHAPES.items():
        dy = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        gw = torch.zeros(N, K, device="cuda")
        gb = torch.zeros(N, K, device="cuda")
        fns = {"tfk": lambda: G.linear_wgrad(dy, x, gw),
               "blas": lambda: torch.ops.aten.mm.dtype_out(dy.t(), x, torch.float32, out=gb)}
        res = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, fn in fns.items():
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) / args.iters * 1000.0)
        fl = 2.0 * M * N * K
        rel = float((gw - gb).norm() / (gb.norm() + 1e-12))
        out = {"shape": name, "N": N, "K": K, "M": M, "rel_diff": round(rel, 6)}
        for k in fns:
            us = statistics.median(res[k])
            out[k + "_us"] = round(us, 1)
            out[k + "_tfs"] = round(fl / us / 1e6, 1)
        print(json.dumps(out), flush=True)
        del dy, x, gw, gb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
