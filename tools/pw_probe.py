#!/usr/bin/env python3
"""Driver for rocprofv3 PMC passes on ResNet-50's memory-bound pointwise GEMMs (bs256 shapes):
the forward 1x1 conv with fused BN statistics, the 1x1 dgrad with the fused BN-backward reduction
(mask + residual), and a stage-3 3x3 forward conv. Runs each a few times on random data.

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -- python3 tools/pw_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops import norm as BN  # noqa: E402


def r(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def main(reps: int = 5):
    M = 256 * 56 * 56
    # forward 1x1 conv a2[M,64] -> y3[M,256] + BN stats
    g = G.ConvGeom(256, 56, 56, 64, 256, 1, 1)
    x, w = r(256, 56, 56, 64), r(256, 1, 1, 64) * 0.1
    st = BN.BNState(256, "cuda")
    # 1x1 dgrad dy[M,64] @ w1[64,256] -> dx[M,256] + BN3 reduce of the previous block (mask, resid)
    gd = G.ConvGeom(256, 56, 56, 256, 64, 1, 1)
    dy, w1 = r(256, 56, 56, 64), r(64, 1, 1, 256) * 0.1
    y3, res = r(256, 56, 56, 256), r(256, 56, 56, 256)
    st3 = BN.BNState(256, "cuda")
    mk = BN.pack_relu_mask(r(256, 56, 56, 256))
    # 3x3 stage 3
    g3 = G.ConvGeom(256, 28, 28, 128, 128, 3, 3, 1, 1, 1, 1)
    x3, w3 = r(256, 28, 28, 128), r(128, 3, 3, 128) * 0.05
    for _ in range(reps):
        G.conv_fwd(x, w, g, st.stats, st.shards)
        G.conv_dgrad(dy, w1, gd, resid=res, bnr=BN.BNReduce(y3, st3, a=mk, premask=True))
        G.conv_fwd(x3, w3, g3)
    torch.cuda.synchronize()
    print("pw_probe done", M)


if __name__ == "__main__":
    main()
