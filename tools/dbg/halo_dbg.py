"""Locate mismatches of the halo conv vs the gather path (debug aid)."""
import sys
import torch
sys.path.insert(0, ".")
from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops._lib import lib

for (N, HW, C) in [(2, 56, 64), (2, 28, 128)]:
    g = G.ConvGeom(N, HW, HW, C, C, 3, 3, 1, 1, 1, 1)
    torch.manual_seed(0)
    x = torch.randn(N, HW, HW, C).to(torch.bfloat16).cuda()
    w = (torch.randn(C, 3, 3, C) * 0.05).to(torch.bfloat16).cuda()
    out = {}
    for halo in (1, 0):
        lib().halo_set(halo)
        st = torch.zeros(16 * 2 * C, device="cuda")
        out[halo] = G.conv_fwd(x, w, g, stats=st, shards=16).float().cpu()
        torch.cuda.synchronize()
    lib().halo_set(-1)
    a, b = out[1], out[0]
    bad = ~torch.isclose(a, b, rtol=2e-2, atol=2e-2)
    print(N, HW, C, "nan", int(torch.isnan(a).sum()), "bad", int(bad.sum()), "of", a.numel())
    if bad.any():
        idx = bad.nonzero()
        print(" n range", idx[:, 0].unique().tolist()[:10], "h", idx[:, 1].unique().tolist()[:60])
        print(" w", idx[:, 2].unique().tolist()[:60], "c", idx[:, 3].unique().tolist()[:70])
        i = idx[0].tolist()
        print(" first", i, float(a[tuple(i)]), float(b[tuple(i)]))
