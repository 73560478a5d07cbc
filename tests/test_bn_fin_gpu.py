"""BN finalize fused into the producing GEMM (ops.norm.BNFinalize, gemm_epilogue.h bn_fin_tail):
the GEMM's last-arriving workgroup reduces the statistics shards. Checked against the standalone
finalize kernels (bn_finalize / bn_bwd_finalize) on the same GEMM output, over the engines the conv
shapes route to (g4 dense / gather, halo 3x3, the register engine's separate-launch fallback,
phased strided dgrads), twice in a row (the tail re-zeroes shards and ticket)."""
import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops import norm as BN
from tensorflow_k8s_amd.ops._lib import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def vec(C, seed, lo=0.5):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(C, generator=g) + lo).to(DEV)


def close(a, b, tol=1e-4):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12)) < tol


FWD = [(2, 8, 8, 64, 256, 1, 1, 1, 0),      # pointwise, g4 dense
       (2, 14, 14, 64, 128, 3, 3, 1, 1),    # 3x3 gather
       (2, 56, 56, 64, 64, 3, 3, 1, 1),     # halo direct conv
       (2, 15, 13, 32, 48, 3, 3, 2, 1),     # ragged: register engine, separate finalize
       (4, 7, 7, 512, 2048, 1, 1, 1, 0)]    # wide output (2048 channels in one tail)


@pytest.mark.parametrize("cfg", FWD)
def test_forward_fused_finalize_matches_standalone(cfg):
    N, H, W, C, K, R, S, s, p = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, s, s, p, p)
    x = bf(N, H, W, C, seed=1)
    w = bf(K, R, S, C, scale=0.05, seed=2)
    gamma, beta = vec(K, 3), vec(K, 4, lo=-0.5)
    M = N * g.P * g.Q
    out = {}
    for fused in (False, True):
        st = BN.BNState(K, DEV)
        rm, rv = torch.zeros(K, device=DEV), torch.ones(K, device=DEV)
        for rep in range(2):
            if fused:
                fin = BN.BNFinalize(st, gamma, beta=beta, eps=1e-5, momentum=0.1, run_mean=rm, run_var=rv)
                y = G.conv_fwd(x, w, g, st.stats, st.shards, fin=fin)
            else:
                y = G.conv_fwd(x, w, g, st.stats, st.shards)
                BN.bn_finalize(st, float(M), gamma, beta, 1e-5, 0.1, rm, rv)
            torch.cuda.synchronize()
            out[(fused, rep)] = [t.clone() for t in (y, st.mean, st.invstd, st.scale, st.shift, rm, rv)]
            assert float(st.stats.abs().max()) == 0.0, "shards re-zeroed for the next accumulation"
            assert int(st.ticket.abs().max()) == 0, "ticket back at rest"
    for rep in range(2):
        a, b = out[(False, rep)], out[(True, rep)]
        assert torch.equal(a[0], b[0])
        for i in range(1, 7):
            assert close(b[i], a[i]), (rep, i)


BWD = [(2, 8, 8, 64, 256, 1, 1, 1, 0),      # pointwise dgrad
       (2, 9, 9, 64, 64, 3, 3, 1, 1),       # stride-1 3x3 (dgrad as forward conv)
       (2, 14, 14, 256, 512, 1, 1, 2, 0),   # strided 1x1 (gather)
       (2, 16, 16, 64, 64, 3, 3, 2, 1),     # strided 3x3: phased, finalize on the last phase
       (2, 15, 13, 32, 48, 3, 3, 2, 1)]     # ragged: register engine fallback


@pytest.mark.parametrize("mode", ["relu_from_y", "dual"])
@pytest.mark.parametrize("cfg", BWD)
def test_backward_fused_finalize_matches_standalone(cfg, mode):
    N, H, W, C, K, R, S, s, p = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, s, s, p, p)
    w = bf(K, R, S, C, scale=0.05, seed=2)
    dy = bf(N, g.P, g.Q, K, seed=3)
    y, y2, a = bf(N, H, W, C, seed=4), bf(N, H, W, C, seed=5), bf(N, H, W, C, seed=6)
    gamma, gamma2 = vec(C, 7), vec(C, 8)
    cnt = N * H * W
    dual = mode == "dual"
    out = {}
    for fused in (False, True):
        st, st2 = BN.BNState(C, DEV), BN.BNState(C, DEV)
        for k, s_ in enumerate((st, st2)):
            s_.mean.copy_(vec(C, 10 + k, lo=-0.5) * 0.1); s_.invstd.copy_(vec(C, 12 + k))
            s_.scale.copy_(vec(C, 14 + k, lo=-0.5)); s_.shift.copy_(vec(C, 16 + k, lo=-0.5) * 0.1)
        dg, db, dg2, db2 = (torch.zeros(C, device=DEV) for _ in range(4))
        for rep in range(2):
            fin = None
            if fused:
                kw = dict(st2=st2, gamma2=gamma2, dgamma2=dg2, dbeta2=db2) if dual else {}
                fin = BN.BNFinalize(st, gamma, dgamma=dg, dbeta=db, count=cnt, **kw)
            spec = (BN.BNReduce(y, st, a=a, y2=y2, st2=st2, fin=fin) if dual else BN.BNReduce(y, st, fin=fin))
            dx = G.conv_dgrad(dy, w, g, bnr=spec)
            if not fused:
                lib().bn_bwd_finalize(st.sums, st.shards, C, float(cnt), gamma, st.mean, st.invstd,
                                      gamma2 if dual else None, st2.mean if dual else None,
                                      st2.invstd if dual else None, dg, db, dg2 if dual else None,
                                      db2 if dual else None, st.coef, st2.coef if dual else None)
            torch.cuda.synchronize()
            out[(fused, rep)] = [t.clone() for t in (dx, dg, db, st.coef, dg2, db2, st2.coef)]
            assert float(st.sums.abs().max()) == 0.0
            assert int(st.ticket.abs().max()) == 0
    for rep in range(2):
        a_, b_ = out[(False, rep)], out[(True, rep)]
        assert torch.equal(a_[0], b_[0])
        for i in range(1, 7 if dual else 4):
            assert close(b_[i], a_[i], 1e-4), (rep, i)
