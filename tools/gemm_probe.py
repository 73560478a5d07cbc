#!/usr/bin/env python3
"""Driver for rocprofv3 PMC passes on the g4 engine's dense GEMM: [M,K] x [N,K]^T bf16 at the
256x256 (16-wave) and 128x128 (4-wave) tiles, a few launches each on random operands.

    rocprofv3 --pmc <counters> -- python3 tools/gemm_probe.py [M N K]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402


def main():
    M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (4096, 4096, 4096)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for t in ((256, 256), (128, 128)):
        for _ in range(5):
            G._gemm(x, w, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, t)
    torch.cuda.synchronize()
    print("gemm_probe done")


if __name__ == "__main__":
    main()
