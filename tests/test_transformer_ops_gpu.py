"""Transformer kernels (attention.hip, transformer.hip, GEMM aux/dact epilogues) vs fp32 PyTorch
references of the same ops."""
import math

import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops import transformer as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def bf(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16)


CASES = [
    # B, H, Sq, Sk, causal, kv_len, p_drop, fused_qkv
    (2, 4, 128, 128, False, None, 0.0, True),
    (2, 3, 100, 100, True, None, 0.0, True),
    (3, 2, 77, 130, False, [130, 64, 1], 0.0, False),
    (2, 2, 64, 192, False, None, 0.1, False),
    (1, 2, 256, 256, True, None, 0.1, True),
]


@pytest.mark.parametrize("case", CASES)
def test_attention_fwd_bwd(case):
    B, H, Sq, Sk, causal, kvl, p, fused = case
    W = H * 64
    if fused:
        assert Sq == Sk
        qkv = bf(B * Sq, 3 * W, seed=1)
        bufs = {"q": (qkv, 0), "k": (qkv, W), "v": (qkv, 2 * W)}
    else:
        bufs = {"q": (bf(B * Sq, W, seed=1), 0), "k": (bf(B * Sk, W, seed=2), 0), "v": (bf(B * Sk, W, seed=3), 0)}
    dout = bf(B * Sq, W, seed=4)
    kv = torch.tensor(kvl, dtype=torch.int32) if kvl else None
    res = {}
    for dev in ("cpu", DEV):
        mv = lambda t: (t[0].to(dev), t[1])
        sp = T.AttnSpec(B, H, Sq, Sk, mv(bufs["q"]), mv(bufs["k"]), mv(bufs["v"]),
                        kv_len=kv.to(dev) if kv is not None else None, causal=causal, p_drop=p, seed=1234)
        out, lse = T.attention_fwd(sp)
        if fused:
            g = torch.zeros(B * Sq, 3 * W, dtype=torch.bfloat16, device=dev)
            dq, dk, dv = (g, 0), (g, W), (g, 2 * W)
        else:
            dq = (torch.zeros(B * Sq, W, dtype=torch.bfloat16, device=dev), 0)
            dk = (torch.zeros(B * Sk, W, dtype=torch.bfloat16, device=dev), 0)
            dv = (torch.zeros(B * Sk, W, dtype=torch.bfloat16, device=dev), 0)
        T.attention_bwd(sp, out, dout.to(dev), lse, dq, dk, dv)
        res[dev] = dict(out=out, lse=lse, dq=dq[0][:, dq[1]:dq[1] + W], dk=dk[0][:, dk[1]:dk[1] + W],
                        dv=dv[0][:, dv[1]:dv[1] + W])
    for k in ("out", "dq", "dk", "dv"):
        assert rel(res[DEV][k], res["cpu"][k]) < 2e-2, k
    finite = torch.isfinite(res["cpu"]["lse"])
    assert torch.allclose(res[DEV]["lse"].cpu()[finite], res["cpu"]["lse"][finite], atol=1e-2)


@pytest.mark.parametrize("n", [8192 * 4, 1001])
def test_dropout_kernel_matches_cpu(n):
    """Standalone dropout (8-wide vector kernel for n % 8 == 0, scalar otherwise) == the CPU hash
    mask bit for bit."""
    from tensorflow_k8s_amd.ops import elementwise as E
    x = bf(n, seed=31)
    assert torch.equal(E.dropout(x.to(DEV), 0.3, 1234).cpu(), E.dropout(x, 0.3, 1234))


def test_linear_dgrad_fused_input_dropout():
    """FFN backward: relu' and the relu-dropout backward fused into the ff2 dgrad epilogue == the
    CPU reference, and == the unfused GEMM + standalone dropout up to one bf16 rounding."""
    from tensorflow_k8s_amd.ops import elementwise as E
    from tensorflow_k8s_amd.ops import gemm as G
    M, N, K = 300, 136, 264
    dy, w, z = bf(M, N, seed=32), bf(N, K, seed=33, scale=0.1), bf(M, K, seed=34)
    ref = G.linear_dgrad(dy, w, dact_src=z, dact="relu", drop_p=0.1, drop_seed=77)
    fused = G.linear_dgrad(dy.to(DEV), w.to(DEV), dact_src=z.to(DEV), dact="relu", drop_p=0.1, drop_seed=77)
    plain = E.dropout(G.linear_dgrad(dy.to(DEV), w.to(DEV), dact_src=z.to(DEV), dact="relu"), 0.1, 77)
    assert rel(fused, ref) < 1e-2
    assert rel(fused, plain) < 1e-2
    assert torch.equal(fused.cpu() == 0, plain.cpu() == 0)


def test_dropout_mask_rate():
    m = T.dropout_keep_mask(7, 2, 3, 64, 64, 0.1)
    assert abs(float(m.float().mean()) - 0.9) < 0.01


@pytest.mark.parametrize("W", [768, 1024, 264])
def test_layernorm(W):
    M = 300
    x = bf(M, W, seed=5, scale=2.0)
    dy = bf(M, W, seed=6)
    dres = bf(M, W, seed=7)
    g = torch.rand(W) + 0.5
    b = torch.randn(W) * 0.1
    out = {}
    for dev in ("cpu", DEV):
        y, mu, rs = T.layernorm_fwd(x.to(dev), g.to(dev), b.to(dev))
        dg, db = torch.zeros(W, device=dev), torch.zeros(W, device=dev)
        dx = T.layernorm_bwd(dy.to(dev), x.to(dev), g.to(dev), mu, rs, dg, db, dres=dres.to(dev))
        out[dev] = dict(y=y, mu=mu, rs=rs, dx=dx, dg=dg, db=db)
    for k in out["cpu"]:
        assert rel(out[DEV][k], out["cpu"][k]) < 1e-2, k


@pytest.mark.parametrize("M,W", [(300, 768), (1000, 1024), (8192, 1024), (17, 1024)])
def test_layernorm_fwd_fast_matches_generic(M, W):
    """The width-specialized LayerNorm forward (transformer.hip ln_fwd_fast_kernel: gamma / beta in
    registers, grid-stride rows; W = 1024, other widths keep ln_fwd_kernel) is bit-identical to
    ln_fwd_kernel: y, mean and rstd."""
    from tensorflow_k8s_amd.ops._lib import lib
    x = bf(M, W, seed=61, scale=2.0).to(DEV)
    g, b = (torch.rand(W) + 0.5).to(DEV), (torch.randn(W) * 0.1).to(DEV)
    out = []
    try:
        for fast in (0, 1):
            lib().ln_fwd_set_fast(fast)
            out.append(T.layernorm_fwd(x, g, b))
    finally:
        lib().ln_fwd_set_fast(1)
    for a, c in zip(*out):
        assert torch.equal(a, c)


@pytest.mark.parametrize("W", [1024, 768, 264])
def test_layernorm_bwd_fused_consumer_dropout(W):
    """LayerNorm backward also emitting dropout(dx) for its consumer: dx unchanged and the second
    output == the standalone dropout of dx, bit for bit (same hash mask, same arithmetic)."""
    from tensorflow_k8s_amd.ops import elementwise as E
    M = 300
    x, dy, dres = bf(M, W, seed=41, scale=2.0), bf(M, W, seed=42), bf(M, W, seed=43)
    g, b = torch.rand(W) + 0.5, torch.randn(W) * 0.1
    y, mu, rs = T.layernorm_fwd(x.to(DEV), g.to(DEV), b.to(DEV))
    outs = []
    for drop in (None, (0.3, 99)):
        dg, db = torch.zeros(W, device=DEV), torch.zeros(W, device=DEV)
        outs.append(T.layernorm_bwd(dy.to(DEV), x.to(DEV), g.to(DEV), mu, rs, dg, db, dres=dres.to(DEV), drop=drop))
    dx, (dx2, dxd) = outs
    assert torch.equal(dx, dx2)
    assert torch.equal(dxd, E.dropout(dx, 0.3, 99))


@pytest.mark.parametrize("W", [768, 1024])
@pytest.mark.parametrize("dres_on,drop_on,dbias_on", [(a, b, c) for a in (0, 1) for b in (0, 1) for c in (0, 1)])
def test_layernorm_bwd_fast_matches_generic(W, dres_on, drop_on, dbias_on):
    """The width-specialized LayerNorm backward (transformer.hip ln_bwd_fast_kernel) == the generic
    kernel for every option combination: dx / dropout(dx) (up to the row reductions' rounding),
    dgamma / dbeta / consumer bias gradient."""
    from tensorflow_k8s_amd.ops._lib import lib
    M = 1000
    x, dy, dres = bf(M, W, seed=51, scale=2.0), bf(M, W, seed=52), bf(M, W, seed=53)
    g, b = torch.rand(W) + 0.5, torch.randn(W) * 0.1
    y, mu, rs = T.layernorm_fwd(x.to(DEV), g.to(DEV), b.to(DEV))
    out = []
    try:
        for fast in (0, 1):
            lib().ln_bwd_set_fast(fast)
            dg, db = torch.zeros(W, device=DEV), torch.zeros(W, device=DEV)
            dbias = torch.zeros(W, device=DEV) if dbias_on else None
            r = T.layernorm_bwd(dy.to(DEV), x.to(DEV), g.to(DEV), mu, rs, dg, db,
                                dres=dres.to(DEV) if dres_on else None, drop=(0.2, 7) if drop_on else None,
                                dbias=dbias)
            dx, dxd = r if drop_on else (r, r)
            out.append((dx, dxd, dg, db, dbias))
    finally:
        lib().ln_bwd_set_fast(1)
    (dx0, dxd0, dg0, db0, bs0), (dx1, dxd1, dg1, db1, bs1) = out
    assert rel(dx1, dx0) < 1e-2 and rel(dxd1, dxd0) < 1e-2
    assert rel(dg1, dg0) < 1e-4 and rel(db1, db0) < 1e-4
    if dbias_on:
        assert rel(bs1, bs0) < 1e-3
    if drop_on:  # the fast kernel's mask is the dropout kernel's, bit for bit
        from tensorflow_k8s_amd.ops import elementwise as E
        assert torch.equal(dxd1, E.dropout(dx1, 0.2, 7))


def test_embedding():
    V, W, S, B = 1000, 768, 128, 4
    word, pos, typ = bf(V, W, seed=8), bf(S, W, seed=9), bf(2, W, seed=10)
    ids = torch.randint(0, V, (B * S,), dtype=torch.int32)
    tt = torch.randint(0, 2, (B * S,), dtype=torch.int32)
    dy = bf(B * S, W, seed=11)
    out = {}
    for dev in ("cpu", DEV):
        o = T.embedding_fwd(ids.to(dev), word.to(dev), pos.to(dev), S, tt.to(dev), typ.to(dev), scale=2.0)
        dw, dp, dt = torch.zeros(V, W, device=dev), torch.zeros(S, W, device=dev), torch.zeros(2, W, device=dev)
        T.embedding_bwd(ids.to(dev), dy.to(dev), dw, dp, S, tt.to(dev), dt, scale=2.0)
        out[dev] = dict(o=o, dw=dw, dp=dp, dt=dt)
    for k in out["cpu"]:
        assert rel(out[DEV][k], out["cpu"][k]) < 1e-2, k


def test_embedding_bwd_replayed_from_a_forked_graph():
    """The bucketed word-row gradient (count -> scan -> scatter -> reduce) captured in a hipGraph whose
    body also forks onto a second stream (as a data-parallel step forks onto the RCCL comm stream),
    replayed 6 times: every replay equals the fp32 reference -- the per-call counts are zeroed by a
    kernel node (a captured hipMemsetAsync was not reliably replayed: round-4 fault, perf_log_r5.md)
    -- and the kernels' out-of-range guard never fires."""
    from tensorflow_k8s_amd.ops._lib import lib
    V, W, ntok = 4096, 256, 2048
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, V, (ntok,), dtype=torch.int32, generator=g)
    dy = bf(ntok, W, seed=12)
    ref = torch.zeros(V, W).index_add_(0, ids.long(), dy.float())
    ids_d, dy_d = ids.to(DEV), dy.to(DEV)
    dw = torch.zeros(V, W, device=DEV)
    side = torch.cuda.Stream()
    lib().emb_guard_count()

    def body():
        dw.zero_()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            torch.cuda._sleep(1000)
        T.embedding_bwd(ids_d, dy_d, dw)
        torch.cuda.current_stream().wait_stream(side)

    for _ in range(2):
        body()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        body()
    for _ in range(6):
        dw.fill_(123.0)  # poison: only a complete replay restores the gradient
        graph.replay()
        torch.cuda.synchronize()
        assert rel(dw, ref) < 1e-2
    assert lib().emb_guard_count() == 0


def test_linear_gelu_aux_and_dact():
    M, K, N = 256, 768, 3072
    x, w = bf(M, K, seed=12), bf(N, K, seed=13, scale=0.03)
    bias = torch.randn(N) * 0.1
    dy = bf(M, N, seed=14)
    w2 = bf(K, N, seed=15, scale=0.03)  # second FFN layer [out=K][in=N]
    out = {}
    for dev in ("cpu", DEV):
        z = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        a = G.linear_fwd(x.to(dev), w.to(dev), bias.to(dev), act="gelu", aux=z)
        # FFN backward: dZ = (dY[M,K] @ W2[K,N]) * gelu'(z), fused in the dgrad epilogue
        dz = G.linear_dgrad(bf(M, K, seed=16).to(dev), w2.to(dev), dact_src=z, dact="gelu")
        # fused dropout after the activation, then residual add; pooler-style tanh
        r = bf(M, N, seed=17)
        ad = G.linear_fwd(x.to(dev), w.to(dev), bias.to(dev), act="gelu", resid=r.to(dev), drop_p=0.1, drop_seed=99)
        th = G.linear_fwd(x.to(dev), w.to(dev), bias.to(dev), act="tanh")
        out[dev] = dict(a=a, z=z, dz=dz, ad=ad, th=th)
    for k in out["cpu"]:
        assert rel(out[DEV][k], out["cpu"][k]) < 1e-2, k


def test_head_row_gather_scatter_match_index_ops():
    """BERT's prediction-head rows (misc.hip gather_rows / scatter_add_rows) against torch's
    index_select / index_add_ in f32: MLM positions (with a repeated position inside a sequence, which
    must accumulate) and the [CLS] rows."""
    B, S, W, P = 6, 40, 768, 7
    g = torch.Generator().manual_seed(5)
    h = torch.randn(B * S, W, generator=g).to(torch.bfloat16)
    pos = torch.randint(1, S, (B, P), generator=g, dtype=torch.int32)
    pos[2, 3] = pos[2, 1]  # repeated position
    rows = (torch.arange(B)[:, None] * S + pos.long()).reshape(-1)
    got = T.gather_rows(h.to(DEV), pos.to(DEV), S)
    assert torch.equal(got.cpu(), h.index_select(0, rows))
    assert torch.equal(T.gather_rows(h.to(DEV), None, S).cpu(), h.index_select(0, torch.arange(B) * S))
    dm = torch.randn(B * P, W, generator=g).to(torch.bfloat16)
    dc = torch.randn(B, W, generator=g).to(torch.bfloat16)
    dh = torch.zeros(B * S, W, dtype=torch.bfloat16, device=DEV)
    T.scatter_add_rows(dh, dm.to(DEV), pos.to(DEV), S)
    T.scatter_add_rows(dh, dc.to(DEV), None, S)
    ref = torch.zeros(B * S, W)
    ref.index_add_(0, rows, dm.float())
    ref.index_add_(0, torch.arange(B) * S, dc.float())
    assert rel(dh.cpu().float(), ref) < 5e-3
