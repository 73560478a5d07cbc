#!/usr/bin/env python3
"""Flash-attention kernel timing (fwd, dQ+dK/dV backward) at the model shapes, with and without
attention dropout: TFLOP/s per pass. python tools/attn_bench.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import transformer as T  # noqa: E402

SHAPES = {"tfm_big_self": (32, 16, 256, 256, False), "tfm_big_causal": (32, 16, 256, 256, True),
          "bert_base": (64, 12, 128, 128, False), "s1024": (8, 16, 1024, 1024, False)}


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    D = T.HEAD_DIM
    for name, (B, H, S, Sk, causal) in SHAPES.items():
        qkv = (torch.randn(B * S, 3 * H * D, device="cuda") * 0.5).to(torch.bfloat16)
        dout = torch.randn(B * S, H * D, device="cuda").to(torch.bfloat16)
        dqkv = torch.empty_like(qkv)
        row = {"shape": name, "B": B, "H": H, "S": S, "causal": causal}
        from tensorflow_k8s_amd.ops._lib import lib
        for p, nw in ((0.0, 4), (0.1, 4), (0.0, 8), (0.1, 8)):
            lib().attn_set_waves(nw)
            sp = T.AttnSpec(B, H, S, Sk, (qkv, 0), (qkv, H * D), (qkv, 2 * H * D), causal=causal, p_drop=p, seed=7)
            out, lse = T.attention_fwd(sp)
            if nw > 4:  # same result as the 4-wave kernels
                lib().attn_set_waves(4)
                o4, l4 = T.attention_fwd(sp)
                lib().attn_set_waves(nw)
                row[f"max_diff_w{nw}_p{p}"] = float((out.float() - o4.float()).abs().max())
            f = 4.0 * B * H * S * Sk * D * (0.5 if causal else 1.0)
            tf = timeit(lambda: T.attention_fwd(sp))
            tb = timeit(lambda: T.attention_bwd(sp, out, dout, lse, (dqkv, 0), (dqkv, H * D), (dqkv, 2 * H * D)))
            row[f"fwd_us_p{p}_w{nw}"] = round(tf * 1e6, 1)
            row[f"bwd_us_p{p}_w{nw}"] = round(tb * 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
