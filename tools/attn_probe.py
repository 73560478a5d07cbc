#!/usr/bin/env python3
"""Driver for rocprofv3 PMC passes on the attention kernels: Transformer-big self-attention shape
(B 32, H 16, S 256, head 64, dropout 0.1), forward + backward, --reps times, no timing.

    rocprofv3 --pmc <counters> -- python3 tools/attn_probe.py [--reps 5] [--causal]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import transformer as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--causal", action="store_true")
    ap.add_argument("--p", type=float, default=0.1)
    args = ap.parse_args()
    B, H, S, D = 32, 16, 256, T.HEAD_DIM
    qkv = (torch.randn(B * S, 3 * H * D, device="cuda") * 0.5).to(torch.bfloat16)
    dout = torch.randn(B * S, H * D, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    sp = T.AttnSpec(B, H, S, S, (qkv, 0), (qkv, H * D), (qkv, 2 * H * D), causal=args.causal, p_drop=args.p, seed=7)
    for _ in range(args.reps):
        out, lse = T.attention_fwd(sp)
        T.attention_bwd(sp, out, dout, lse, (dqkv, 0), (dqkv, H * D), (dqkv, 2 * H * D))
    torch.cuda.synchronize()
    print("attn_probe done")


if __name__ == "__main__":
    main()
