"""T5 kernel numerics: every gfx950 HIP kernel against the fp32 torch reference of the same op
(the CPU path of each ops module), on random data, over the ResNet/BERT shape envelope plus
ragged tails. Runs only on a real MI355X; the native library must be the thing under test."""
import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops import loss as LS
from tensorflow_k8s_amd.ops import norm as BN
from tensorflow_k8s_amd.ops import optim as O
from tensorflow_k8s_amd.ops import pool as PL
from tensorflow_k8s_amd.ops._lib import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16)


def test_native_loaded():
    L = lib()
    assert hasattr(L, "gemm") and L.__file__.endswith(".so")


CONVS = [
    # N, H, W, C, K, R, S, stride, pad
    (2, 8, 8, 64, 256, 1, 1, 1, 0),
    (2, 9, 9, 64, 64, 3, 3, 1, 1),
    (2, 16, 16, 128, 128, 3, 3, 2, 1),
    (2, 14, 14, 256, 512, 1, 1, 2, 0),
    (2, 32, 32, 8, 64, 7, 7, 2, 3),
    (3, 7, 7, 24, 40, 3, 3, 1, 1),
    (1, 5, 6, 16, 200, 3, 3, 2, 1),
    # Cout <= 64 non-pointwise weight gradients take the 64x256 tile (stem 7x7 on C padded to 8, ragged M/N)
    (1, 20, 20, 8, 64, 7, 7, 2, 3),
    (1, 10, 10, 16, 48, 3, 3, 1, 1),
    # stride-1 dgrads with >= 128 input channels run as a forward conv over dY (flipped weights, g4)
    (2, 9, 9, 128, 64, 3, 3, 1, 1),
    (1, 12, 12, 128, 64, 5, 5, 1, 2),
    (2, 10, 10, 256, 128, 3, 3, 1, 1),
    (1, 9, 11, 128, 64, 3, 3, 1, 0),
]


@pytest.mark.parametrize("cfg", CONVS)
def test_conv_fwd_dgrad_wgrad(cfg):
    N, H, W, C, K, R, S, st, pd = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, st, st, pd, pd)
    x = bf(N, H, W, C, seed=1)
    w = bf(K, R, S, C, scale=0.05, seed=2)
    stats_ref = torch.zeros(2 * K)
    y_ref = G.conv_fwd(x, w, g, stats_ref, 1)
    stats = torch.zeros(4 * 2 * K, device=DEV)
    y = G.conv_fwd(x.to(DEV), w.to(DEV), g, stats, 4)
    assert y.shape == y_ref.shape
    assert rel(y, y_ref) < 1e-2
    s = stats.view(4, 2, K).sum(0).cpu()
    assert rel(s[0], stats_ref.view(2, K)[0]) < 1e-3
    assert rel(s[1], stats_ref.view(2, K)[1]) < 1e-3
    dy = bf(*y_ref.shape, seed=3)
    resid = bf(N, H, W, C, seed=4)
    dx_ref = G.conv_dgrad(dy, w, g, resid=resid)
    dx = G.conv_dgrad(dy.to(DEV), w.to(DEV), g, resid=resid.to(DEV))
    assert rel(dx, dx_ref) < 1e-2
    gw_ref = torch.zeros(K, R, S, C)
    G.conv_wgrad(dy, x, g, gw_ref)
    gw = torch.zeros(K, R, S, C, device=DEV)
    G.conv_wgrad(dy.to(DEV), x.to(DEV), g, gw)
    assert rel(gw, gw_ref) < 5e-3
    # accumulate path
    G.conv_wgrad(dy.to(DEV), x.to(DEV), g, gw, accumulate=True)
    assert rel(gw, 2 * gw_ref) < 5e-3


@pytest.mark.parametrize("cfg", [(2, 9, 9, 64, 64, 3, 3, 1, 1), (1, 20, 20, 8, 64, 7, 7, 2, 3),
                                 (1, 10, 10, 16, 48, 3, 3, 1, 1), (2, 12, 12, 32, 64, 3, 3, 2, 1)])
def test_conv_wgrad_wide_tile(cfg, monkeypatch):
    """The 64x256 weight-gradient tile (forced; the picker only takes it at ResNet-scale K)."""
    N, H, W, C, K, R, S, st, pd = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, st, st, pd, pd)
    x = bf(N, H, W, C, seed=1)
    dy = bf(N, g.P, g.Q, K, seed=3)
    gw_ref = torch.zeros(K, R, S, C)
    G.conv_wgrad(dy, x, g, gw_ref)
    monkeypatch.setattr(G, "pick_tile", lambda *a, **k: (64, 256))
    for splits in (1, 3):
        gw = torch.zeros(K, R, S, C, device=DEV)
        G.conv_wgrad(dy.to(DEV), x.to(DEV), g, gw, splits=splits)
        assert rel(gw, gw_ref) < 5e-3, splits


@pytest.mark.parametrize("M,K,N", [(37, 64, 200), (256, 2048, 1000), (512, 768, 3072), (128, 3072, 768), (8, 16, 24)])
def test_linear(M, K, N):
    x = bf(M, K, seed=5)
    w = bf(N, K, scale=0.05, seed=6)
    b = torch.randn(N)
    for act in (None, "relu", "gelu"):
        y_ref = G.linear_fwd(x, w, b, act=act)
        y = G.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), act=act)
        assert rel(y, y_ref) < 1e-2, act
    dy = bf(M, N, seed=7)
    if K % 8 == 0:
        assert rel(G.linear_dgrad(dy.to(DEV), w.to(DEV)), G.linear_dgrad(dy, w)) < 1e-2
    if N % 8 == 0 and K % 8 == 0:
        gw_ref = torch.zeros(N, K)
        G.linear_wgrad(dy, x, gw_ref)
        gw = torch.zeros(N, K, device=DEV)
        G.linear_wgrad(dy.to(DEV), x.to(DEV), gw)
        assert rel(gw, gw_ref) < 5e-3
    gb_ref = torch.zeros(N)
    G.bias_grad(dy, gb_ref)
    gb = torch.zeros(N, device=DEV)
    G.bias_grad(dy.to(DEV), gb)
    assert rel(gb, gb_ref) < 1e-3


@pytest.mark.parametrize("M,N,ld", [(8192, 768, 768), (8192, 3072, 3072), (100, 520, 520), (33, 24, 40), (70, 13, 13)])
def test_bias_grad_colsum(M, N, ld):
    """Column sums: 16-B vector path (N, ld multiples of 8) and the scalar fallback; write + accumulate."""
    full = bf(M, ld, seed=11)
    dy = full[:, :N].contiguous()
    ref = dy.float().sum(0)
    gb = torch.zeros(N, device=DEV)
    lib().colsum(full.to(DEV), M, N, ld, gb)  # strided rows: only the first N of each ld are summed
    assert rel(gb, ref) < 1e-4
    G.bias_grad(dy.to(DEV), gb, accumulate=True)
    assert rel(gb, 2 * ref) < 1e-4


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C write (cdna_hip_programming.md §3)."""
    n = 64
    eye = torch.eye(n).to(torch.bfloat16)
    B = torch.arange(n * n, dtype=torch.float32).reshape(n, n).remainder(17).to(torch.bfloat16)
    y = G.linear_fwd(eye.to(DEV), B.to(DEV))  # = I @ B^T
    assert torch.equal(y.cpu().float(), B.float().t())


@pytest.mark.parametrize("C", [64, 24])  # 24: C does not divide 2048 -> flat (non-fixed-chunk) kernels
@pytest.mark.parametrize("proj", [False, True])
def test_bn_fused_forward_backward(proj, C):
    N, H, W = 4, 10, 10
    M = N * H * W
    y = bf(N, H, W, C, seed=8)
    y2 = bf(N, H, W, C, seed=9)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    gamma2, beta2 = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    out = {}
    for dev in ("cpu", DEV):
        st, st2 = BN.BNState(C, dev), BN.BNState(C, dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        BN.bn_stats(y.to(dev), st)
        BN.bn_finalize(st, M, gamma.to(dev), beta.to(dev), 1e-5, 0.1, rm, rv)
        r = y2.to(dev)
        if proj:
            BN.bn_stats(r, st2)
            BN.bn_finalize(st2, M, gamma2.to(dev), beta2.to(dev), 1e-5, 0.1, None, None)
        a = BN.bn_apply(y.to(dev), st, True, r=r, rst=st2 if proj else None)
        da = bf(N, H, W, C, seed=10).to(dev)
        dg, db, dg2, db2 = (torch.zeros(C, device=dev) for _ in range(4))
        dy, dy2, dres = BN.bn_backward(da, a, y.to(dev), st, gamma.to(dev), dg, db, M,
                                       y2=r if proj else None, st2=st2 if proj else None,
                                       gamma2=gamma2.to(dev) if proj else None, dgamma2=dg2, dbeta2=db2,
                                       want_dres=not proj)
        out[dev] = dict(a=a, dy=dy, dy2=dy2, dres=dres, dg=dg, db=db, dg2=dg2, rm=rm, rv=rv)
        # relu mask recomputed from y (no residual input): a = relu(bn(y))
        a1 = BN.bn_apply(y.to(dev), st, True)
        dg3, db3 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dy3, _, _ = BN.bn_backward(da, None, y.to(dev), st, gamma.to(dev), dg3, db3, M, relu_from_y=True)
        out[dev].update(a1=a1, dy3=dy3, dg3=dg3, db3=db3)
    for k, v in out["cpu"].items():
        if v is None:
            continue
        assert rel(out[DEV][k], v) < 1e-2, k


@pytest.mark.parametrize("C", [64, 256, 192])
@pytest.mark.parametrize("proj", [False, True])
def test_bn_finalize_in_apply_matches_separate(proj, C, monkeypatch):
    """The finalize-in-apply BN passes (bn.hip bn_apply_fin / bn_bwd_apply_fin, pooled states,
    ops/norm.py FUSED_FIN) equal the separate finalize + apply kernels: activations, relu bitmask,
    saved mean/invstd/scale/shift, running statistics, input gradients (incl. the projection-shortcut
    BN and the identity residual) and dgamma/dbeta -- for the tensor-mask and relu-from-y backwards.
    Ragged row counts (M not a multiple of a block's rows) included."""
    N, H, W = 3, 11, 13
    M = N * H * W
    y, r = bf(N, H, W, C, seed=31).to(DEV), bf(N, H, W, C, seed=32).to(DEV)
    da = bf(N, H, W, C, seed=33).to(DEV)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.1).to(DEV)
    gamma2, beta2 = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.1).to(DEV)
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(BN, "FUSED_FIN", fused)
        pool = BN.BNPool([C, C], DEV)
        st, st2 = pool.states
        pool.zero()
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        BN.bn_stats(y, st)
        BN.bn_finalize(st, M, gamma, beta, 1e-5, 0.1, rm, rv, defer=True)
        if proj:
            BN.bn_stats(r, st2)
            BN.bn_finalize(st2, M, gamma2, beta2, 1e-5, 0.1, None, None, defer=True)
        assert (st.fin is not None) == fused
        a, mk = BN.bn_apply(y, st, True, r=r, rst=st2 if proj else None, mask=True)
        dg, db, dg2, db2 = (torch.zeros(C, device=DEV) for _ in range(4))
        dy, dy2, dres = BN.bn_backward(da, mk, y, st, gamma, dg, db, M, y2=r if proj else None,
                                       st2=st2 if proj else None, gamma2=gamma2 if proj else None, dgamma2=dg2,
                                       dbeta2=db2, want_dres=not proj)
        pool.zero()
        dg3, db3 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        dy3, _, _ = BN.bn_backward(da, None, y, st, gamma, dg3, db3, M, relu_from_y=True)
        torch.cuda.synchronize()
        res[fused] = dict(a=a, mk=mk, mean=st.mean.clone(), invstd=st.invstd.clone(), scale=st.scale.clone(),
                          shift=st.shift.clone(), rm=rm, rv=rv, dy=dy, dy2=dy2, dres=dres, dg=dg, db=db, dg2=dg2,
                          db2=db2, dy3=dy3, dg3=dg3, db3=db3)
    for k, v in res[False].items():
        if v is None:
            assert res[True][k] is None, k
            continue
        if v.dtype == torch.uint8:
            assert (res[True][k] != v).float().mean() < 1e-3, k  # a bf16 tie may round the other way
        else:
            assert rel(res[True][k], v) < 1e-3, k


@pytest.mark.parametrize("proj", [False, True])
def test_bn_relu_bitmask(proj):
    """bn_apply(mask=True) writes the packed relu mask of its output (bit e of byte i = a[8i+e] > 0),
    and the BN backward / fused dgrad reduction driven by that bitmask equal the bf16-a versions
    bit for bit (the ResNet tail reads 1 bit per element instead of a)."""
    C, N, H, W = 256, 4, 9, 7
    M = N * H * W
    y, r = bf(N, H, W, C, seed=21).to(DEV), bf(N, H, W, C, seed=22).to(DEV)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.1).to(DEV)
    st, st2 = BN.BNState(C, DEV), BN.BNState(C, DEV)
    for s_ in (st, st2):
        BN.bn_stats(y if s_ is st else r, s_)
        BN.bn_finalize(s_, M, gamma, beta, 1e-5, 0.1, None, None)
    a, mk = BN.bn_apply(y, st, True, r=r, rst=st2 if proj else None, mask=True)
    assert mk.dtype == torch.uint8 and mk.numel() == a.numel() // 8
    assert torch.equal(mk, BN.pack_relu_mask(a))
    assert torch.equal(BN.unpack_relu_mask(mk.cpu(), a.shape), a.cpu().float() > 0)
    da = bf(N, H, W, C, seed=23).to(DEV)
    outs = []
    for m in (a, mk):
        dg, db, dg2, db2 = (torch.zeros(C, device=DEV) for _ in range(4))
        outs.append(BN.bn_backward(da, m, y, st, gamma, dg, db, M, y2=r if proj else None,
                                   st2=st2 if proj else None, gamma2=gamma if proj else None, dgamma2=dg2,
                                   dbeta2=db2, want_dres=not proj) + (dg, db))
    for u, v in zip(*outs):
        assert (u is None and v is None) or torch.equal(u, v)
    # fused into a dgrad epilogue: packed mask vs the CPU oracle on the bf16 activation
    g = G.ConvGeom(N, H, W, C, 64, 1, 1, 1, 1, 0, 0)
    w, dy = bf(64, 1, 1, C, scale=0.05, seed=24).to(DEV), bf(N, H, W, 64, seed=25).to(DEV)
    st.sums.zero_()
    dx = G.conv_dgrad(dy, w, g, bnr=BN.BNReduce(y, st, a=mk))
    ref = BN.BNState(C, "cpu")
    ref.mean.copy_(st.mean.cpu()); ref.invstd.copy_(st.invstd.cpu())
    BN.BNReduce(y.cpu(), ref, a=a.cpu()).reference_accumulate(dx.cpu())
    got = st.sums.view(st.shards, 3, C).sum(0).cpu()
    for k in range(2):
        assert rel(got[k], ref.sums.view(1, 3, C)[0, k]) < 2e-2, k


@pytest.mark.parametrize("mode", ["relu_from_y", "mask_a", "none"])
@pytest.mark.parametrize("C", [64, 32, 256])
def test_maxpool_bwd_fused_bn_reduce(mode, C):
    """Max-pool backward with the producer BN's backward reduction fused in (the ResNet stem):
    dx unchanged, channel sums == the fp32 CPU oracle (BNReduce.reference_accumulate)."""
    x = bf(2, 17, 19, C, seed=21)
    y = bf(2, 17, 19, C, seed=22)
    a = bf(2, 17, 19, C, seed=23)
    gen = torch.Generator().manual_seed(24)
    mu, inv = torch.randn(C, generator=gen) * 0.1, torch.rand(C, generator=gen) + 0.5
    sc, sh = torch.randn(C, generator=gen), torch.randn(C, generator=gen) * 0.1
    res = {}
    for dev in ("cpu", DEV):
        _, idx = PL.maxpool_fwd(x.to(dev))
        dy = bf(2, 9, 10, C, seed=25).to(dev)
        st = BN.BNState(C, dev)
        st.mean.copy_(mu); st.invstd.copy_(inv); st.scale.copy_(sc); st.shift.copy_(sh)
        spec = BN.BNReduce(y.to(dev), st, a=a.to(dev) if mode == "mask_a" else None, relu=mode != "none")
        dx = PL.maxpool_bwd(dy, idx, x.shape, bnr=spec)
        plain = PL.maxpool_bwd(dy, idx, x.shape)
        res[dev] = (dx.cpu(), plain.cpu(), st.sums.view(st.shards, 3, C).sum(0).cpu())
    assert torch.equal(res[DEV][0], res[DEV][1])
    assert rel(res[DEV][0], res["cpu"][0]) < 1e-2
    for k in range(2):
        assert rel(res[DEV][2][k], res["cpu"][2][k]) < 2e-2, k


def test_pools():
    x = bf(2, 17, 17, 64, seed=11)
    y_ref, idx_ref = PL.maxpool_fwd(x)
    y, idx = PL.maxpool_fwd(x.to(DEV))
    assert torch.equal(y.cpu(), y_ref)
    dy = bf(*y.shape, seed=12)
    assert rel(PL.maxpool_bwd(dy.to(DEV), idx, x.shape), PL.maxpool_bwd(dy, idx_ref, x.shape)) < 1e-2
    assert rel(PL.avgpool_fwd(x.to(DEV)), PL.avgpool_fwd(x)) < 1e-2
    g = bf(2, 64, seed=13)
    assert rel(PL.avgpool_bwd(g.to(DEV), x.shape), PL.avgpool_bwd(g, x.shape)) < 1e-2


@pytest.mark.parametrize("C", [64, 24])
def test_maxpool_fused_bn_relu_equals_separate(C):
    """maxpool_fwd(y, bn=(scale, shift)) -- the stem BN + relu applied inside the pool -- equals the
    pool over the materialized bn_apply output bit for bit (values and argmax bytes), and the CPU
    reference of the fused form."""
    y = bf(3, 23, 19, C, seed=41).to(DEV)
    scale = (torch.rand(C) * 2 - 0.5).to(DEV)  # some negative: the BN may flip the order
    shift = (torch.randn(C) * 0.3).to(DEV)
    st = BN.BNState(C, DEV)
    st.scale.copy_(scale); st.shift.copy_(shift)
    a = BN.bn_apply(y, st, relu=True)
    p_ref, i_ref = PL.maxpool_fwd(a, 3, 2, 1)
    p, i = PL.maxpool_fwd(y, 3, 2, 1, bn=(scale, shift))
    assert torch.equal(p, p_ref) and torch.equal(i, i_ref)
    p_cpu, _ = PL.maxpool_fwd(y.cpu(), 3, 2, 1, bn=(scale.cpu(), shift.cpu()))
    assert rel(p, p_cpu) < 1e-2  # the CPU reference rounds x*scale+shift without an FMA


@pytest.mark.parametrize("B,V,smooth", [(64, 1000, 0.1), (33, 30522, 0.0), (16, 37, 0.1)])
def test_softmax_xent(B, V, smooth):
    x = bf(B, V, scale=3.0, seed=14)
    lab = torch.randint(0, V, (B,), dtype=torch.int32)
    lab[0] = -100
    l_ref, d_ref, c_ref = LS.softmax_xent(x, lab, smooth, scale=1.0 / B, want_correct=True)
    l, d, c = LS.softmax_xent(x.to(DEV), lab.to(DEV), smooth, scale=1.0 / B, want_correct=True)
    assert rel(l, l_ref) < 1e-3
    assert rel(d, d_ref) < 1e-2
    assert torch.equal(c.cpu(), c_ref)


def test_optimizers():
    n = 10007
    w = torch.randn(n); g = torch.randn(n); m = torch.randn(n) * 0.1; v = torch.rand(n) * 0.1
    wc, mc = w.clone(), m.clone()
    O.sgd_(wc, None, g, mc, 0.1, 0.9, 1e-4, True, 0.5)
    wg, mg, wb = w.to(DEV), m.to(DEV), torch.empty(n, dtype=torch.bfloat16, device=DEV)
    O.sgd_(wg, wb, g.to(DEV), mg, 0.1, 0.9, 1e-4, True, 0.5)
    assert rel(wg, wc) < 1e-6 and rel(mg, mc) < 1e-6 and rel(wb, wc) < 1e-2
    wc, mc, vc = w.clone(), m.clone(), v.clone()
    O.adamw_(wc, None, g, mc, vc, 1e-3, 0.9, 0.999, 1e-6, 0.01, 3)
    wg, mg, vg = w.to(DEV), m.to(DEV), v.to(DEV)
    O.adamw_(wg, None, g.to(DEV), mg, vg, 1e-3, 0.9, 0.999, 1e-6, 0.01, 3)
    assert rel(wg, wc) < 1e-6 and rel(vg, vc) < 1e-6


@pytest.mark.parametrize("n,off", [(10007, 0), (1 << 20, 0), (4099, 1), (3, 0)])
def test_adamw_vector_and_tail(n, off):
    """AdamW: 4-wide vector kernel + scalar tail (n % 4), the misaligned fallback (off=1), bf16 shadow."""
    w = torch.randn(n + off); g = torch.randn(n + off); m = torch.randn(n + off) * 0.1; v = torch.rand(n + off) * 0.1
    wc, mc, vc = w[off:].clone(), m[off:].clone(), v[off:].clone()
    O.adamw_(wc, None, g[off:], mc, vc, 1e-3, 0.9, 0.98, 1e-9, 0.01, 7)
    wg, mg, vg, gg = w.to(DEV), m.to(DEV), v.to(DEV), g.to(DEV)
    wb = torch.empty(n + off, dtype=torch.bfloat16, device=DEV)
    O.adamw_(wg[off:], wb[off:], gg[off:], mg[off:], vg[off:], 1e-3, 0.9, 0.98, 1e-9, 0.01, 7)
    assert rel(wg[off:], wc) < 1e-6 and rel(mg[off:], mc) < 1e-6 and rel(vg[off:], vc) < 1e-6
    assert rel(wb[off:], wc) < 1e-2
    if off:
        assert float(wg[0].cpu()) == float(w[0])  # element before the slice untouched


@pytest.mark.parametrize("B,V,ld,smooth", [(24, 33708, 33712, 0.1), (8, 33708, 33728, 0.1), (8, 8195, 8200, 0.0), (16, 32000, 32000, 0.1),
                                          (4, 40960, 40960, 0.0)])
def test_softmax_xent_padded_vocab(B, V, ld, smooth):
    """Register-resident xent kernel: vocab padded to ld (the Transformer-big 33708 -> 33712 layout),
    padding columns excluded from the softmax and given a zero gradient; argmax ties / ignore_index."""
    x = bf(B, ld, scale=3.0, seed=15)
    x[1, 5] = x[1, 9] = 40.0  # tie: smallest index wins
    lab = torch.randint(0, V, (B,), dtype=torch.int32)
    lab[0] = -100
    lab[1] = 5
    l_ref, d_ref, c_ref = LS.softmax_xent(x, lab, smooth, scale=1.0 / B, want_correct=True, V=V)
    l, d, c = LS.softmax_xent(x.to(DEV), lab.to(DEV), smooth, scale=1.0 / B, want_correct=True, V=V)
    assert rel(l, l_ref) < 1e-3
    assert rel(d[:, :V], d_ref[:, :V]) < 1e-2
    assert float(d[:, V:].float().abs().sum().cpu()) == 0.0
    assert torch.equal(c.cpu(), c_ref)


def test_global_norm_clip():
    g = torch.randn(100000) * 3
    ss, coef, nrm = (torch.zeros(1, device=DEV) for _ in range(3))
    O.global_norm_clip_coef(g.to(DEV), 1.0, ss, coef, nrm)
    assert abs(float(nrm) - float(g.norm())) / float(g.norm()) < 1e-4
    assert abs(float(coef) - 1.0 / float(g.norm())) < 1e-5


@pytest.mark.parametrize("mode", ["relu_from_y", "mask_a", "dual"])
@pytest.mark.parametrize("cfg", [(2, 8, 8, 64, 256, 1, 1, 1, 0), (2, 9, 9, 64, 64, 3, 3, 1, 1), (2, 14, 14, 256, 512, 1, 1, 2, 0),
                                 (2, 16, 16, 64, 64, 3, 3, 2, 1), (2, 15, 13, 32, 48, 3, 3, 2, 1),
                                 (2, 9, 9, 128, 64, 3, 3, 1, 1), (3, 20, 20, 256, 256, 3, 3, 1, 1),
                                 (2, 14, 14, 64, 128, 3, 3, 2, 1), (2, 15, 13, 64, 128, 3, 3, 2, 1),
                                 (2, 12, 12, 32, 64, 5, 5, 2, 2)])
def test_dgrad_fused_bn_reduce(cfg, mode):
    """BN-backward channel sums fused into the dgrad epilogue == the standalone reduction."""
    N, H, W, C, K, R, S, st_, pd = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, st_, st_, pd, pd)
    w = bf(K, R, S, C, scale=0.05, seed=2)
    dy = bf(N, g.P, g.Q, K, seed=3)
    y = bf(N, H, W, C, seed=4)
    y2 = bf(N, H, W, C, seed=5)
    a = bf(N, H, W, C, seed=6)
    gen = torch.Generator().manual_seed(7)
    stat_vals = [(torch.randn(C, generator=gen) * 0.1, torch.rand(C, generator=gen) + 0.5,
                  torch.randn(C, generator=gen), torch.randn(C, generator=gen) * 0.1) for _ in range(2)]
    res = {}
    for dev in ("cpu", DEV):
        st, st2 = BN.BNState(C, dev), BN.BNState(C, dev)
        for s_, (mu, inv, sc, sh) in zip((st, st2), stat_vals):
            s_.mean.copy_(mu); s_.invstd.copy_(inv); s_.scale.copy_(sc); s_.shift.copy_(sh)
        if mode == "relu_from_y":
            spec = BN.BNReduce(y.to(dev), st)
        elif mode == "mask_a":
            spec = BN.BNReduce(y.to(dev), st, a=a.to(dev))
        else:
            spec = BN.BNReduce(y.to(dev), st, a=a.to(dev), y2=y2.to(dev), st2=st2)
        dx = G.conv_dgrad(dy.to(dev), w.to(dev), g, bnr=spec)
        res[dev] = (dx, st.sums.view(st.shards, 3, C).sum(0).cpu())
    assert rel(res[DEV][0], res["cpu"][0]) < 1e-2
    for k in range(3 if mode == "dual" else 2):
        assert rel(res[DEV][1][k], res["cpu"][1][k]) < 2e-2, k


@pytest.mark.parametrize("mode", ["relu_from_y", "mask_a", "dual"])
@pytest.mark.parametrize("cfg", [(2, 9, 9, 64, 64, 3, 3, 1, 1), (3, 20, 20, 64, 128, 3, 3, 1, 1)])
def test_dgrad_as_fwd_256x64(cfg, mode, monkeypatch):
    """64-channel stride-1 dgrad as a forward conv on g4's 4-wave 256x64 gather tile with the fused
    BN-backward reduction (ResNet stage-1 3x3): same checks as test_dgrad_fused_bn_reduce."""
    monkeypatch.setattr(G, "DGRAD_AS_FWD_MIN_C", 64)
    monkeypatch.setattr(G, "FORCE_TILE", (256, 64))
    assert G.dgrad_as_fwd_geom(G.ConvGeom(*cfg[:7], cfg[7], cfg[7], cfg[8], cfg[8])) is not None
    test_dgrad_fused_bn_reduce(cfg, mode)


@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (520, 300, 200), (777, 1030, 136)])
def test_big_tile_256(M, N, K, monkeypatch):
    """The 8-wave 256x256 tile (dense operand modes) on interior and ragged shapes: fwd (bias+gelu
    with aux) and dgrad (K-outer B, fused GELU backward); wgrad (split-K) stays on 128 tiles."""
    real = G.pick_tile
    monkeypatch.setattr(G, "pick_tile", lambda m, n, splits_ok=False, big_ok=False, K=0, **kw:
                        (256, 256) if big_ok and not splits_ok and m >= 256 and n >= 256
                        else real(m, n, splits_ok, big_ok, K, **kw))
    x, w = bf(M, K, seed=1), bf(N, K, seed=2, scale=0.05)
    b = torch.randn(N) * 0.1
    dy = bf(M, N, seed=3)
    w2 = bf(K, N, seed=4, scale=0.05)
    out = {}
    for dev in ("cpu", DEV):
        z = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        y = G.linear_fwd(x.to(dev), w.to(dev), b.to(dev), act="gelu", aux=z)
        dz = G.linear_dgrad(bf(M, K, seed=5).to(dev), w2.to(dev), dact_src=z, dact="gelu")
        dx = G.linear_dgrad(dy.to(dev), w.to(dev))
        gw = torch.zeros(N, K, device=dev)
        G.linear_wgrad(dy.to(dev), x.to(dev), gw)
        out[dev] = dict(y=y, z=z, dz=dz, dx=dx, gw=gw)
    for k in out["cpu"]:
        assert rel(out[DEV][k], out["cpu"][k]) < 1e-2, k


@pytest.mark.parametrize("M,N,K", [(70001, 256, 64), (40000, 64, 256), (33000, 200, 136)])
def test_persistent_gemm_matches_one_shot(M, N, K):
    """Far more tiles than resident blocks -> persistent grid (next tile prefetched during the
    epilogue). Must equal the one-shot grid bitwise (same per-tile math) and the fp32 reference."""
    L = lib()
    x, w = bf(M, K, seed=1), bf(N, K, scale=0.05, seed=2)
    xd, wd = x.to(DEV), w.to(DEV)
    res = {}
    try:
        for flag in (0, 1):
            L.gemm_set_persist(flag)
            y = G.linear_fwd(xd, wd, act="relu")
            dx = G.linear_dgrad(y, wd) if N % 8 == 0 else None
            res[flag] = (y, dx)
    finally:
        L.gemm_set_persist(1)
    assert torch.equal(res[0][0], res[1][0])
    if res[1][1] is not None:
        assert torch.equal(res[0][1], res[1][1])
    assert rel(res[1][0], G.linear_fwd(x, w, act="relu")) < 1e-2


def test_persistent_conv_stats():
    """Pointwise conv fwd on a persistent grid: output and fused BN batch statistics."""
    g = G.ConvGeom(64, 32, 32, 64, 256, 1, 1)
    x = bf(64, 32, 32, 64, seed=3)
    w = bf(256, 1, 1, 64, scale=0.05, seed=4)
    st_ref = torch.zeros(2 * 256)
    y_ref = G.conv_fwd(x, w, g, st_ref, 1)
    st = torch.zeros(32 * 2 * 256, device=DEV)
    y = G.conv_fwd(x.to(DEV), w.to(DEV), g, st, 32)
    assert rel(y, y_ref) < 1e-2
    s = st.view(32, 2, 256).sum(0).cpu()
    assert rel(s[0], st_ref.view(2, 256)[0]) < 1e-3
    assert rel(s[1], st_ref.view(2, 256)[1]) < 1e-3


@pytest.mark.parametrize("mode", ["mask_a", "dual"])
def test_dgrad_lattice_resid(mode):
    """Pointwise dgrad + a stride-2 sub-sampled residual (the strided projection shortcut's
    lattice gradient) with the fused BN reduction, against the CPU reference."""
    N, H, W, C, K = 2, 14, 13, 64, 128
    g = G.ConvGeom(N, H, W, C, K, 1, 1)
    w = bf(K, 1, 1, C, scale=0.05, seed=2)
    dy = bf(N, H, W, K, seed=3)
    t = bf(N, (H + 1) // 2, (W + 1) // 2, C, seed=4)
    y, y2, a = bf(N, H, W, C, seed=5), bf(N, H, W, C, seed=6), bf(N, H, W, C, seed=7)
    gen = torch.Generator().manual_seed(8)
    vals = [(torch.randn(C, generator=gen) * 0.1, torch.rand(C, generator=gen) + 0.5) for _ in range(2)]
    res = {}
    for dev in ("cpu", DEV):
        st, st2 = BN.BNState(C, dev), BN.BNState(C, dev)
        for s_, (mu, inv) in zip((st, st2), vals):
            s_.mean.copy_(mu); s_.invstd.copy_(inv)
        spec = BN.BNReduce(y.to(dev), st, a=a.to(dev), y2=y2.to(dev) if mode == "dual" else None,
                           st2=st2 if mode == "dual" else None)
        dx = G.conv_dgrad(dy.to(dev), w.to(dev), g, resid=t.to(dev), bnr=spec, resid_stride=2)
        res[dev] = (dx, st.sums.view(st.shards, 3, C).sum(0).cpu())
    assert rel(res[DEV][0], res["cpu"][0]) < 1e-2
    for k in range(3 if mode == "dual" else 2):
        assert rel(res[DEV][1][k], res["cpu"][1][k]) < 2e-2, k


@pytest.mark.parametrize("M,N,K", [(64, 256, 200704), (256, 1152, 50176), (100, 72, 30000)])
def test_splitk_slab_wgrad_matches_fp32(M, N, K):
    """Weight-gradient-shaped GEMMs (tiny M x N, huge K -> hundreds of split-K slabs + the
    deterministic reduce) agree with fp32, overwriting and accumulating."""
    dy, x = bf(K, M, seed=3), bf(K, N, seed=4)
    ref = dy.float().t() @ x.float()
    gw = torch.full((M, N), 7.0, device=DEV)
    G.linear_wgrad(dy.to(DEV), x.to(DEV), gw)
    acc = torch.ones(M, N, device=DEV)
    G.linear_wgrad(dy.to(DEV), x.to(DEV), acc, accumulate=True)
    assert rel(gw.cpu(), ref) < 1e-3
    assert rel(acc.cpu(), ref + 1.0) < 1e-3


G4_SHAPES = [(256, 256, 64), (512, 768, 1024), (300, 264, 200), (1000, 520, 72), (2048, 1024, 136),
             (4200, 4104, 200)]  # last: 289 tiles > 256 resident blocks -> persistent multi-item walk


@pytest.mark.parametrize("tile", [(256, 256), (128, 128), (256, 128), (128, 256), "g8"])
@pytest.mark.parametrize("M,N,K", G4_SHAPES)
def test_lds_dma_gemm_modes(M, N, K, tile):
    """The LDS-DMA GEMM engines in every dense mode they serve: NT bf16 (bias+relu), NN bf16
    (residual), TN f32 (beta accumulate; split-K slabs), on interior and ragged M/N/K (zero-filled
    out-of-range DMA), against the fp32 reference AND the register-staged engine: gemm_g4.hip's
    64x64 wave tiles (256x256 = 16 waves, 128x128 = 4; the 8-wave 3-stage 256x128 / 128x256) and
    "g8", gemm_g8.hip's 8-phase 256x256 schedule (quadrant wave layout, counted vmcnt)."""
    L = lib()
    if tile == "g8":
        L.g8_set(1)
        tile = (256, 256)
    else:
        L.g8_set(0)
    x, w = bf(M, K, seed=1), bf(N, K, seed=2, scale=0.05)
    dy, r = bf(M, N, seed=3), bf(M, K, seed=4)
    b = torch.randn(N) * 0.1
    gw0 = torch.randn(N, K)
    xd, wd, dyd, rd, bd = x.to(DEV), w.to(DEV), dy.to(DEV), r.to(DEV), b.to(DEV)
    t = tile
    engines = (1, 0)
    res = {}
    try:
        for eng in engines:
            L.gemm_set_engine(eng)
            y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
            G._gemm(xd, wd, y, M, N, K, K, K, N, G.A_KIN, G.B_KIN, G.EPI_BF16, t, bias=bd, act=1)
            dx = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
            G._gemm(dyd, wd, dx, M, K, N, N, K, K, G.A_KIN, G.B_KOUT, G.EPI_BF16, t, resid=rd)
            gw = gw0.clone().to(DEV)
            G._gemm(dyd, xd, gw, N, K, M, N, K, K, G.A_KOUT, G.B_KOUT, G.EPI_F32, t, beta=1.0)
            ns = int(L.gemm_splits(M, 3))
            stride = ((N * K + 3) // 4) * 4
            ws = torch.full((ns * stride,), float("nan"), device=DEV)
            G._gemm(dyd, xd, ws, N, K, M, N, K, K, G.A_KOUT, G.B_KOUT, G.EPI_F32, t, splits=3, split_stride=stride)
            gws = ws.view(ns, stride)[:, :N * K].sum(0).view(N, K)
            torch.cuda.synchronize()
            res[eng] = dict(y=y, dx=dx, gw=gw, gws=gws)
    finally:
        L.gemm_set_engine(1)
        L.g8_set(0)
    ref = dict(y=torch.relu(x.float() @ w.float().t() + b),
               dx=(dy.float() @ w.float()).to(torch.bfloat16).float() + r.float(),
               gw=gw0 + dy.float().t() @ x.float(), gws=dy.float().t() @ x.float())
    for k, v in ref.items():
        for eng in engines[:-1]:
            assert rel(res[eng][k], v) < 1e-2, (eng, k, rel(res[eng][k], v))
            assert rel(res[eng][k], res[0][k]) < 1e-2, (eng, k)


@pytest.mark.parametrize("cfg", [(2, 14, 14, 64, 128, 3, 3, 1, 1), (3, 9, 11, 128, 200, 3, 3, 2, 1),
                                 (2, 8, 8, 64, 64, 1, 1, 2, 0), (1, 30, 30, 64, 136, 5, 5, 1, 2),
                                 # Cin < 64: several taps per K-tile (stem 7x7/2 on 8 channels, ragged K)
                                 (2, 20, 20, 8, 64, 7, 7, 2, 3), (1, 15, 17, 16, 72, 3, 3, 1, 1),
                                 (2, 9, 9, 32, 64, 5, 5, 2, 2)])
@pytest.mark.parametrize("tile", [(256, 256), (128, 128), (256, 64), "g8"])
def test_g4_conv_fwd_gather(cfg, tile):
    """g4's implicit-GEMM conv-forward gather (Cin % 64 == 0: a K-tile is one tap x 64 channels;
    Cin % 8 == 0 below 64: 64/Cin taps per K-tile; zero padding from out-of-range DMA) against the
    fp32 reference, with BN statistics."""
    N, H, W, C, K, R, S, st, pd = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, st, st, pd, pd)
    x, w = bf(N, H, W, C, seed=7), bf(K, R, S, C, scale=0.05, seed=8)
    M = N * g.P * g.Q
    Kd = R * S * C
    y = torch.empty(N, g.P, g.Q, K, dtype=torch.bfloat16, device=DEV)
    st_ = torch.zeros(2, K, device=DEV)
    g8 = tile == "g8"  # gemm_g8.hip's 8-phase engine (Cin % 64 == 0 convs; others fall back to g4)
    lib().g8_set(1 if g8 else 0)
    try:
        G._gemm(x.to(DEV), w.to(DEV), y, M, K, Kd, 0, Kd, K, G.A_CONV_FWD, G.B_KIN, G.EPI_BF16,
                (256, 256) if g8 else tile, stats=st_, shards=1, conv=g.vec())
    finally:
        lib().g8_set(0)
    ref = G._ref_conv(x, w, g)
    assert rel(y, ref) < 1e-2
    assert rel(st_[0], ref.reshape(-1, K).sum(0)) < 1e-2


@pytest.mark.parametrize("shape", [(4, 28, 28, 64, 256), (3, 17, 19, 64, 200), (4, 28, 28, 256, 128),
                                   (3, 17, 19, 192, 200), (2, 14, 14, 512, 256)])
def test_shortk_single_stage_blocks(shape):
    """Few-K-tile GEMMs (1x1 convs with 64..512 input channels, 1..8 K-tiles of 64): the
    single-stage 4-blocks-per-CU g4 instantiation (looping its K-tiles through one LDS stage) must
    equal the two-stage kernel (same per-tile math) for conv fwd + BN stats and for the BN-reduce
    dgrad, and match the fp32 CPU reference. 128x128 tiles forced (the variant's only tile)."""
    L = lib()
    N, H, W, C, K = shape
    g = G.ConvGeom(N, H, W, C, K, 1, 1)
    x = bf(N, H, W, C, seed=1)
    w = bf(K, 1, 1, C, scale=0.05, seed=2)
    dyk = bf(N, H, W, K, seed=3)            # gradient wrt the K-channel output
    wt = bf(C, 1, 1, K, scale=0.05, seed=4)  # a K -> C conv whose dgrad has K_gemm = C = 64
    g2 = G.ConvGeom(N, H, W, K, C, 1, 1)
    y, a = bf(N, H, W, K, seed=5), bf(N, H, W, K, seed=6)
    gen = torch.Generator().manual_seed(8)
    mu, inv = torch.randn(K, generator=gen) * 0.1, torch.rand(K, generator=gen) + 0.5

    def run(dev):
        st = torch.zeros(8 * 2 * K, device=dev)
        yf = G.conv_fwd(x.to(dev), w.to(dev), g, st, 8)
        bst = BN.BNState(K, dev)
        bst.mean.copy_(mu); bst.invstd.copy_(inv)
        spec = BN.BNReduce(y.to(dev), bst, a=a.to(dev))
        dx = G.conv_dgrad(bf(N, H, W, C, seed=7).to(dev), wt.to(dev), g2, bnr=spec)
        return yf, st.view(8, 2, K).sum(0).cpu(), dx, bst.sums.view(bst.shards, 3, K).sum(0).cpu()

    res = {}
    try:
        G.FORCE_TILE = (128, 128)
        for flag in (0, 8):
            L.gemm_set_shortk(flag)
            res[flag] = run(DEV)
            torch.cuda.synchronize()
    finally:
        G.FORCE_TILE = None
        L.gemm_set_shortk(-1)  # back to the TFK_G4_SHORTK / built-in default
    ref = run("cpu")
    assert torch.equal(res[0][0], res[8][0]) and torch.equal(res[0][2], res[8][2])
    for i in range(4):
        assert rel(res[8][i], ref[i]) < 2e-2, i
        assert rel(res[8][i], res[0][i]) < 1e-4, i


@pytest.mark.parametrize("S,n", [(1, 1000), (3, 4096), (8, 1048576), (256, 16384), (126, 65536), (502, 4100), (5, 1001),
                                 (7, 2359296)])
@pytest.mark.parametrize("acc", [False, True])
def test_splitk_reduce_two_pass(S, n, acc):
    """Split-K slab reduce (misc.hip): deterministic two-pass tree vs an fp64 sum; f32 and bf16
    outputs, accumulate on/off, ragged n (not a multiple of 4), hundreds of slabs."""
    from tensorflow_k8s_amd.ops._lib import lib
    torch.manual_seed(S + n)
    stride = (n + 3) // 4 * 4
    slabs = torch.randn(S * stride, device="cuda")
    ref = slabs.view(S, stride)[:, :n].double().sum(0) * 0.5
    base = torch.randn(n, device="cuda")
    out = base.clone() if acc else torch.full((n,), float("nan"), device="cuda")
    lib().splitk_reduce(slabs.clone(), S, stride, n, out, None, acc, 0.5)
    exp = ref + (base.double() if acc else 0)
    assert float((out.double() - exp).abs().max()) < 1e-3 * (S ** 0.5)
    # bitwise deterministic across calls
    out2 = base.clone() if acc else torch.zeros(n, device="cuda")
    lib().splitk_reduce(slabs.clone(), S, stride, n, out2, None, acc, 0.5)
    assert torch.equal(out, out2)
    if n % 4 == 0:
        ob = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
        lib().splitk_reduce(slabs.clone(), S, stride, n, None, ob, False, 0.5)
        assert float((ob.double() - ref).abs().max()) < 0.02 * float(ref.abs().max()) + 1e-2


@pytest.mark.parametrize("S,n", [(1, 4097), (2, 4194304), (3, 1048579), (4, 2050), (6, 1048576), (8, 262147)])
@pytest.mark.parametrize("mode", [1, 2])
def test_splitk_direct_matches_two_pass(S, n, mode):
    """The S <= 8 one-pass slab reduce (misc.hip splitk_direct_kernel) is bit-identical to the
    two-pass kernel wherever that one runs a single slab group (S <= 4 or >= 1024 chunks): f32
    accumulate and bf16 outputs, ragged n, partial last block, both column counts per lane."""
    from tensorflow_k8s_amd.ops._lib import lib
    L = lib()
    torch.manual_seed(S * 7 + n)
    stride = (n + 3) // 4 * 4
    slabs = torch.randn(S * stride, device="cuda")
    base = torch.randn(n, device="cuda")
    try:
        res = {}
        for m in (0, mode):
            L.splitk_set_direct(m)
            out = base.clone()
            L.splitk_reduce(slabs.clone(), S, stride, n, out, None, True, 0.5)
            ob = torch.full((n,), 3.0, dtype=torch.bfloat16, device="cuda")
            L.splitk_reduce(slabs.clone(), S, stride, n, None, ob, False, 1.0)
            res[m] = (out, ob)
    finally:
        L.splitk_set_direct(2)
    assert torch.equal(res[0][0], res[mode][0])
    assert torch.equal(res[0][1], res[mode][1])


@pytest.mark.parametrize("N,K,M", [(4352, 4096, 2048), (4300, 4096, 1024)])
def test_wgrad_tail_split_matches_reference(N, K, M):
    """Weight gradients of whole 256x256 rounds plus a small tail (272 tiles = 256 + 16): the tail
    row-tiles run split-K into slabs (ops.gemm._wgrad_tail_split); overwrite and accumulate both
    equal the fp32 reference, ragged tail included."""
    dy, x = bf(M, N, seed=5).to(DEV), bf(M, K, seed=6).to(DEV)
    gw = torch.full((N, K), float("nan"), device=DEV)
    G.linear_wgrad(dy, x, gw)
    ref = dy.float().t() @ x.float()
    assert rel(gw, ref) < 1e-4
    G.linear_wgrad(dy, x, gw, accumulate=True)
    assert rel(gw, 2 * ref) < 1e-4


@pytest.mark.parametrize("M,K,N", [(8192, 1024, 33728), (1024, 264, 8192)])
def test_dgrad_splitk_matches_reference(M, K, N):
    """Plain input gradients on the split-K path (few 256x256 output tiles, long reduction: the
    tied-logits dgrad shape and a ragged one): f32 slabs + one bf16 reduce equal the fp32 reference."""
    dy, w = bf(M, N, seed=3).to(DEV), bf(N, K, scale=0.05, seed=4).to(DEV)
    dx = G.linear_dgrad(dy, w)
    ref = dy.float() @ w.float()
    assert rel(dx, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(8192, 4096, 1024), (1000, 264, 128)])
def test_relu_mask_aux_matches_bf16_aux(M, N, K):
    """EXT epilogue with a uint8 relu-mask aux / dact_src (aux_bits, dact_bits) against the bf16
    pre-activation path on the same operands: identical forward outputs, mask = (z > 0) bit for bit,
    identical fused relu(+dropout) backward -- interior tiles and ragged edges."""
    x, w, b = bf(M, K, seed=1).to(DEV), bf(N, K, scale=0.05, seed=2).to(DEV), torch.randn(N).to(DEV)
    z = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    m = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8)
    y1 = G.linear_fwd(x, w, b, act="relu", aux=z, drop_p=0.1, drop_seed=7)
    y2 = G.linear_fwd(x, w, b, act="relu", aux=m, drop_p=0.1, drop_seed=7)
    assert torch.equal(y1, y2)
    assert torch.equal(m.cpu(), G.relu_mask_pack(z.float().cpu()))
    dy, w2 = bf(M, K, seed=3).to(DEV), bf(K, N, scale=0.05, seed=4).to(DEV)
    d1 = G.linear_dgrad(dy, w2, dact_src=z, dact="relu", drop_p=0.1, drop_seed=7)
    d2 = G.linear_dgrad(dy, w2, dact_src=m, dact="relu", drop_p=0.1, drop_seed=7)
    assert torch.equal(d1, d2)


@pytest.mark.parametrize("M,N,K", [(8192, 4096, 1024), (1000, 264, 128)])
def test_dgrad_fused_column_sums(M, N, K):
    """linear_dgrad(colsum=...) accumulates the column sums of the stored dx (the consumer layer's
    bias gradient) in the EXT epilogue: matches dx.sum(0) of the same call, interior and ragged tiles."""
    dy, w = bf(M, K, seed=3).to(DEV), bf(K, N, scale=0.05, seed=4).to(DEV)
    x, w1 = bf(M, 64, seed=5).to(DEV), bf(N, 64, scale=0.1, seed=6).to(DEV)
    m = torch.empty(M, N // 8, device=DEV, dtype=torch.uint8)
    G.linear_fwd(x, w1, act="relu", aux=m)
    cs = torch.full((N,), 0.5, device=DEV)
    dx = G.linear_dgrad(dy, w, dact_src=m, dact="relu", drop_p=0.1, drop_seed=9, colsum=cs)
    ref = dx.float().sum(0) + 0.5
    assert float((cs - ref).abs().max()) <= 1e-3 * float(ref.abs().max()) + 1e-4


@pytest.mark.parametrize("act", ["relu", "gelu"])
@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (300, 200, 136)])
def test_linear_activated_bf16_epilogue(M, N, K, act):
    """An activated bf16 GEMM output without the EXT extras (no aux / dropout) runs the EPI_BF16_ACT
    epilogue -- EPI_BF16's own accumulator pass is activation-free (gemm_epilogue.h)."""
    x, w = bf(M, K, seed=1), bf(N, K, seed=2, scale=0.05)
    b = torch.randn(N) * 0.1
    ref = G.linear_fwd(x, w, b, act=act)
    got = G.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), act=act)
    assert rel(got, ref) < 1e-2


@pytest.mark.parametrize("cfg", [(2, 8, 8, 64, 128, 1, 1, 1, 0), (2, 9, 9, 64, 64, 3, 3, 1, 1), (2, 12, 12, 8, 16, 5, 5, 1, 2)])
def test_conv_relu_bf16_epilogue(cfg):
    """conv + bias + relu (no BatchNorm: LeNet's form) on the activated bf16 epilogue."""
    N, H, W, C, K, R, S, st_, pd = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, st_, st_, pd, pd)
    x, w = bf(N, H, W, C, seed=3), bf(K, R, S, C, seed=4, scale=0.05)
    b = torch.randn(K) * 0.1
    ref = G.conv_fwd(x, w, g, bias=b, act="relu")
    got = G.conv_fwd(x.to(DEV), w.to(DEV), g, bias=b.to(DEV), act="relu")
    assert rel(got, ref) < 1e-2
    assert float(got.float().min()) >= 0.0
