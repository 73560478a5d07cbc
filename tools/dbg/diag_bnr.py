import sys, torch
sys.path.insert(0, '.')
from tensorflow_k8s_amd.ops import gemm as G, norm as BN
from tensorflow_k8s_amd.ops._lib import lib
L = lib()
def bf(*s, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed); return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).cuda()
for (M, N, K) in [(70000, 256, 320), (2000, 256, 320), (70000, 128, 128)]:
    w = bf(N, K, seed=2, scale=0.05); dy = bf(M, N, seed=3); r = bf(M, K, seed=4)
    y2, a2 = bf(M, K, seed=7), bf(M, K, seed=8)
    out = {}
    for flag in (0, 1):
        L.gemm_set_g4_persist(flag)
        st = BN.BNState(K, "cuda"); torch.manual_seed(0); st.mean.uniform_(-0.1, 0.1); st.invstd.uniform_(0.5, 1.5)
        spec = BN.BNReduce(y2.view(M, 1, 1, K), st, a=a2.view(M, 1, 1, K))
        g = G.ConvGeom(M, 1, 1, K, N, 1, 1)
        G.FORCE_TILE = (128, 128)
        dx = G.conv_dgrad(dy.view(M, 1, 1, N), w.view(N, 1, 1, K), g, resid=r.view(M, 1, 1, K), bnr=spec)
        G.FORCE_TILE = None
        torch.cuda.synchronize()
        sums = st.sums.view(st.shards, 3, K).sum(0)
        dz = dx.view(M, K).float() * (a2.float() > 0)
        ref0 = dz.sum(0); ref1 = (dz * (y2.float() - st.mean) * st.invstd).sum(0)
        out[flag] = sums
        print(M, N, K, "persist", flag, "r0 err", float((sums[0] - ref0).norm() / ref0.norm()), "r1 err", float((sums[1] - ref1).norm() / ref1.norm()), flush=True)
L.gemm_set_g4_persist(0)
