"""MX-fp8 quantizer and block-scaled MFMA GEMM (csrc/kernels/fp8.hip) vs exact references:
the quantizer against torch.float8_e4m3fn rounding of the same scaled values, the GEMM against
the fp32 product of the dequantized operands (the MFMA accumulates exactly in f32)."""
import pytest
import torch

from tensorflow_k8s_amd.ops import fp8 as F8

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_quantizer_matches_reference():
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(300, 256, generator=g) * torch.logspace(-3, 2, 256)).to(torch.bfloat16)
    x[5, :32] = 0  # all-zero block
    qc, sc = F8.mx_quantize(x)
    qg, sg = F8.mx_quantize(x.cuda())
    assert torch.equal(sg.cpu(), sc)
    mism = (qg.cpu() != qc).float().mean().item()
    assert mism < 1e-3, mism  # identical up to rare round-to-nearest ties
    assert rel(F8.mx_dequantize(qg, sg), x.float()) < 0.04


@pytest.mark.parametrize("M,N,K", [(128, 128, 128), (256, 384, 512), (300, 200, 1024)])
def test_mx_gemm_exact_integers(M, N, K):
    """Small integers are exact in e4m3 with scale 1 per block -> the GEMM must match exactly;
    any lane/K mapping or scale-operand mistake shows up as a large error."""
    g = torch.Generator().manual_seed(M + N)
    x = torch.randint(-8, 9, (M, K), generator=g).to(torch.bfloat16)
    w = torch.randint(-8, 9, (N, K), generator=g).to(torch.bfloat16)
    x[:, :32] *= 16  # a second scale exponent in the first block of every row
    y = F8.linear_fwd_mx(x.cuda(), w.cuda()).float().cpu()
    ref = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    assert torch.equal(y, ref) or rel(y, ref) < 1e-3


@pytest.mark.parametrize("M,N,K", [(512, 1024, 1024), (200, 300, 256)])
def test_mx_linear_epilogues(M, N, K):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.03).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    r = torch.randn(M, N, generator=g).to(torch.bfloat16)
    out = {}
    for dev in ("cpu", "cuda"):
        z = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        y = F8.linear_fwd_mx(x.to(dev), w.to(dev), b.to(dev), act="relu", aux=z, drop_p=0.1, drop_seed=5,
                             resid=r.to(dev))
        out[dev] = (y, z)
    assert rel(out["cuda"][0], out["cpu"][0]) < 1e-2
    assert rel(out["cuda"][1], out["cpu"][1]) < 1e-2
    # fp8 vs bf16 GEMM: MX-e4m3 quantization error only
    yb = x.float() @ w.float().t() + b
    assert rel(out["cuda"][1].float(), yb) < 0.06


def test_transposed_quantizer_matches_reference():
    """mx_quant_t(x) == mx_quant(x^T): same scales, same bytes up to rounding ties; ragged C."""
    g = torch.Generator().manual_seed(1)
    x = (torch.randn(256, 300, generator=g) * torch.logspace(-2, 1, 300)).to(torch.bfloat16)
    x[:32, 7] = 0
    qc, sc = F8.mx_quantize(x.t().contiguous())
    qg, sg = F8.mx_quantize_t(x.cuda())
    assert qg.shape == (300, 256) and sg.shape == (300, 8)
    assert torch.equal(sg.cpu(), sc)
    assert (qg.cpu() != qc).float().mean().item() < 1e-3


@pytest.mark.parametrize("M,N,K", [(512, 1024, 768), (256, 384, 200)])
def test_mx_dgrad_wgrad(M, N, K):
    """Backward GEMMs on MX-fp8: dX = dY W (W^T quantized along N) with GELU-backward and residual
    epilogue, dW (+)= dY^T X (both quantized along the tokens, f32 accumulate): GPU == the CPU
    dequantized reference, and within MX-e4m3 error of the bf16 products."""
    g = torch.Generator().manual_seed(4)
    dy = torch.randn(M, N, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    z = torch.randn(M, K, generator=g).to(torch.bfloat16)
    r = torch.randn(M, K, generator=g).to(torch.bfloat16)
    gw0 = torch.randn(N, K, generator=g)
    out = {}
    for dev in ("cpu", "cuda"):
        dx = F8.linear_dgrad_mx(dy.to(dev), w.to(dev), resid=r.to(dev), dact_src=z.to(dev), dact="gelu")
        gw = gw0.clone().to(dev)
        F8.linear_wgrad_mx(dy.to(dev), x.to(dev), gw, accumulate=True)
        gw2 = torch.empty(N, K, device=dev)
        F8.linear_wgrad_mx(dy.to(dev), x.to(dev), gw2)
        out[dev] = (dx, gw, gw2)
    for a, b in zip(out["cuda"], out["cpu"]):
        assert rel(a, b) < 1e-2
    from tensorflow_k8s_amd.ops.gemm import act_grad_ref
    dx_ref = (dy.float() @ w.float()) * act_grad_ref(z.float(), "gelu") + r.float()
    assert rel(out["cuda"][0], dx_ref) < 0.06
    assert rel(out["cuda"][2], dy.float().t() @ x.float()) < 0.06


def test_fp8_training_tracks_bf16_200_steps():
    """A tiny Transformer with every linear GEMM on MX-fp8 (fwd + dgrad + wgrad) trains like the
    bf16 model: 200 Adam steps on a fixed batch, loss curves within 3 % (mean over the last 20
    steps) and both converge. The fp8 run takes every producer-emitted MX path (LayerNorm+MX,
    EXT_MX epilogues, grouped weight quantization: 256 tokens tile every GEMM)."""
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    from tensorflow_k8s_amd.runtime.optimizer import AdamW
    curves = {}
    for fp8 in (False, True):
        c = TransformerConfig.tiny()
        c.ffn, c.src_len, c.tgt_len = 512, 32, 32  # 8 x 32 = 256 tokens: every wgrad tiles (M % 128)
        c.dropout = c.attn_dropout = c.relu_dropout = 0.0
        c.fp8 = fp8
        m = Transformer(c).to("cuda", seed=9)
        opt = AdamW(m.arena, lr=1e-3, b2=0.98, eps=1e-9, weight_decay=0.0)
        batch = m.synthetic_batch(8, "cuda", seed=2)
        ls = []
        for _ in range(200):
            loss, _ = m.forward_backward(*batch)
            opt.step()
            ls.append(float(loss.float().mean()))
        curves[fp8] = ls
    b, f = curves[False], curves[True]
    assert all(v == v for v in f), "fp8 loss went NaN"
    assert b[-1] < 0.5 * b[0] and f[-1] < 0.5 * f[0], (b[::20], f[::20])
    mb, mf = sum(b[-20:]) / 20, sum(f[-20:]) / 20
    print(f"fp8 vs bf16 loss, mean of last 20 steps: {mf:.4f} vs {mb:.4f} (gap {abs(mf - mb) / mb:.2%})")
    assert abs(mf - mb) <= 0.03 * mb + 0.02, (b[::20], f[::20])


def test_fp8_real_width_tracks_bf16_100_steps():
    """Transformer-big at its real widths (d 1024, FFN 4096, heads 16, the 33708-entry vocabulary)
    with 1 encoder + 1 decoder layer, dropout ON (0.3 / 0.1 / 0.1, same per-step masks in both
    runs), 100 AdamW steps on a fixed 8 x 256-token batch: MX-fp8 (every linear GEMM fwd + dgrad +
    wgrad, incl. the tied-embedding logits) tracks bf16: mean loss of the last 20 steps within 2.5 %
    (measured r4: 3.229 vs 3.165, 2.03 %, while both memorise the batch from 15.8 down to ~3.2; the
    curves agree to < 0.6 % over the first 50 steps)."""
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    from tensorflow_k8s_amd.runtime.optimizer import AdamW
    curves = {}
    for fp8 in (False, True):
        c = TransformerConfig.big()
        c.enc_layers = c.dec_layers = 1
        c.fp8 = fp8
        m = Transformer(c).to("cuda", seed=11)
        opt = AdamW(m.arena, lr=3e-4, b2=0.98, eps=1e-9, weight_decay=0.0)
        batch = m.synthetic_batch(8, "cuda", seed=3)
        ls = []
        for _ in range(100):
            loss, _ = m.forward_backward(*batch)
            opt.step()
            ls.append(float(loss.float().mean()))
        curves[fp8] = ls
        del m, opt, batch
        torch.cuda.empty_cache()
    b, f = curves[False], curves[True]
    assert all(v == v for v in f), "fp8 loss went NaN"
    assert b[-1] < 0.9 * b[0] and f[-1] < 0.9 * f[0], (b[::10], f[::10])
    mb, mf = sum(b[-20:]) / 20, sum(f[-20:]) / 20
    print(f"real-width fp8 vs bf16 loss, mean of last 20 steps: {mf:.4f} vs {mb:.4f} (gap {abs(mf - mb) / mb:.2%})")
    assert abs(mf - mb) <= 0.025 * mb, (b[::10], f[::10])


def test_fp8_bf16_weight_gradients_finite_and_track_mx_wgrad(monkeypatch):
    """Transformer-big (6+6 layers, real widths, dropout on) in fp8 with bf16 weight gradients
    (ops.fp8.MX_WGRAD False, bench.py --mx-wgrad 0): 20 AdamW steps stay finite and the mean loss is
    within 2 % of the MX-fp8-weight-gradient run. Round 5 shipped this path with ff1's weight
    gradient reading a never-stored bf16 dz (NaN loss)."""
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    from tensorflow_k8s_amd.ops import fp8 as F8
    from tensorflow_k8s_amd.runtime.optimizer import AdamW
    curves = {}
    for mxw in (True, False):
        monkeypatch.setattr(F8, "MX_WGRAD", mxw)
        c = TransformerConfig.big()
        c.fp8 = True
        m = Transformer(c).to("cuda", seed=11)
        opt = AdamW(m.arena, lr=3e-4, b2=0.98, eps=1e-9, weight_decay=0.0)
        batch = m.synthetic_batch(8, "cuda", seed=3)
        ls = []
        for _ in range(20):
            loss, _ = m.forward_backward(*batch)
            opt.step()
            ls.append(float(loss.float().mean()))
        assert torch.isfinite(m.arena.master).all()
        curves[mxw] = ls
        del m, opt, batch
        torch.cuda.empty_cache()
    a, b = curves[True], curves[False]
    assert all(v == v and abs(v) != float("inf") for v in a + b), (a, b)
    ma, mb = sum(a) / len(a), sum(b) / len(b)
    print(f"fp8 loss, MX vs bf16 weight gradients, mean of 20 steps: {ma:.4f} vs {mb:.4f}")
    assert abs(ma - mb) <= 0.02 * ma, (a, b)


@pytest.mark.parametrize("tile", [128, 256, 2561])
@pytest.mark.parametrize("M,N,K", [(512, 1024, 1024), (300, 200, 256), (1000, 520, 384)])
def test_g4_fp8_engine_matches_register_engine(M, N, K, tile):
    """The LDS-DMA (g4) MX-fp8 kernel and the register-staged one run the same quantized operands
    through the same scaled MFMAs in the same K order: results agree to f32 rounding, for the bf16
    (bias/relu/residual), EXT (GELU-backward) and f32 (accumulate) epilogues, incl. ragged M/N, on
    every g4 tile (128x128 4-wave, 256x256 16-wave and 256x128 8-wave blocks -- tile code 2561;
    scales staged by LDS-DMA)."""
    from tensorflow_k8s_amd.ops._lib import lib
    g = torch.Generator().manual_seed(7)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).cuda()
    b = (torch.randn(N, generator=g) * 0.1).cuda()
    r = torch.randn(M, N, generator=g).to(torch.bfloat16).cuda()
    z = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    dy = torch.randn(M, N, generator=g).to(torch.bfloat16).cuda()
    out = {}
    try:
        lib().fp8_set_tile(tile)
        for eng in (1, 0):
            lib().fp8_set_engine(eng)
            y = F8.linear_fwd_mx(x, w, b, act="relu", resid=r)
            dx = F8.linear_dgrad_mx(dy, w, dact_src=z, dact="gelu") if N % 128 == 0 else None
            gw = torch.ones(N, K, device="cuda")
            if M % 128 == 0:
                F8.linear_wgrad_mx(dy, x, gw, accumulate=True)
            torch.cuda.synchronize()
            out[eng] = (y, dx, gw)
    finally:
        lib().fp8_set_engine(-1)
        lib().fp8_set_tile(-1)
    for a, c in zip(out[1], out[0]):
        if a is not None:
            assert rel(a, c) < 1e-5, rel(a, c)


@pytest.mark.parametrize("R,C", [(256, 1024), (4096, 96), (96, 4128)])
def test_dual_quantizer_matches_row_and_transposing_quantizers(R, C):
    """mx_quantize_dual (one read of x) produces bit-identical bytes and scales to mx_quantize(x)
    and mx_quantize_t(x) (ragged column tiles included)."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(R, C, generator=g) * torch.logspace(-3, 3, C)).to(torch.bfloat16).cuda()
    (q, s), (qt, st) = F8.mx_quantize_dual(x)
    q1, s1 = F8.mx_quantize(x)
    qt1, st1 = F8.mx_quantize_t(x)
    torch.cuda.synchronize()
    assert torch.equal(q, q1) and torch.equal(s, s1)
    assert torch.equal(qt, qt1) and torch.equal(st, st1)


def test_dual_quantizer_zero_and_tiny_blocks():
    """All-zero blocks (scale byte 0, bytes 0) and blocks of tiny values (e4m3 subnormal outputs) come
    out of the scaled-convert quantizer exactly as from the multiply-then-convert row quantizer."""
    g = torch.Generator().manual_seed(9)
    x = torch.randn(256, 256, generator=g)
    x[:32, :] = 0
    x[:, 64:96] = 0
    x[100:132, 128:160] *= 1e-30
    x[200:, 200:] *= torch.logspace(-6, 0, 56)
    x = x.to(torch.bfloat16).cuda()
    (q, s), (qt, st) = F8.mx_quantize_dual(x)
    q1, s1 = F8.mx_quantize(x)
    qt1, st1 = F8.mx_quantize_t(x)
    torch.cuda.synchronize()
    assert torch.equal(q, q1) and torch.equal(s, s1)
    assert torch.equal(qt, qt1) and torch.equal(st, st1)
    assert int(s[0, 0]) == 0 and int(q[:32].abs().sum()) == 0


def test_group_quantizer_matches_per_tensor_dual():
    """GroupQuantizer (one launch over a descriptor table, resident blocks walking every tensor's
    tiles) == mx_quantize_dual of each tensor, bit for bit, for mixed / ragged shapes; the results are
    registered for linear_fwd_mx (pre-quantized weight + the saved MX(w^T) for the dgrad)."""
    g = torch.Generator().manual_seed(11)
    shapes = [(256, 1024), (96, 4128), (4096, 96), (128, 128), (1024, 1024), (32, 32), (33792 // 8, 1024)]
    ws = [(torch.randn(*sh, generator=g) * 0.05).to(torch.bfloat16).cuda() for sh in shapes]
    gq = F8.GroupQuantizer(ws)
    F8.clear_saved()
    gq.run()
    torch.cuda.synchronize()
    for w, ((q, s), (qt, st)) in zip(ws, gq.out):
        (q1, s1), (qt1, st1) = F8.mx_quantize_dual(w)
        assert torch.equal(q, q1) and torch.equal(s, s1), w.shape
        assert torch.equal(qt, qt1) and torch.equal(st, st1), w.shape
    # the pre-quantized weight is used by the forward: same output as quantizing on the fly
    x = torch.randn(256, 1024, generator=g).to(torch.bfloat16).cuda()
    y_pre = F8.linear_fwd_mx(x, ws[4], save=True)
    assert F8.take_t(ws[4]) is gq.out[4][1]
    F8.clear_saved()
    y_fly = F8.linear_fwd_mx(x, ws[4])
    torch.cuda.synchronize()
    assert torch.equal(y_pre, y_fly)
    F8.clear_saved()


@pytest.mark.parametrize("M,N,K", [(512, 1024, 1024), (288, 320, 256), (4096, 4096, 1024)])
def test_mx_epilogue_outputs_equal_dual_quantizer(M, N, K):
    """EPI_BF16_EXT_MX: the fp8 GEMM's epilogue writes MX(y) and MX(y^T) from its LDS tile -- the
    same bytes and scales as mx_quantize_dual of the bf16 y it stores (relu + aux + dropout forward;
    relu-backward + dropout dgrad), ragged tiles included; with mx_skip_c the MX copies are unchanged
    and the consumers take them (no bf16 read)."""
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).cuda()
    b = (torch.randn(N, generator=g) * 0.1).cuda()
    z = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    F8.clear_saved()
    y = F8.linear_fwd_mx(x, w, b, act="relu", aux=z, drop_p=0.1, drop_seed=3, mx_out=True)
    c = F8.cached_dual(y)
    assert c is not None
    (q1, s1), (qt1, st1) = F8.mx_quantize_dual(y)
    torch.cuda.synchronize()
    (q, s), (qt, st) = c
    assert torch.equal(q, q1) and torch.equal(s, s1)
    assert torch.equal(qt, qt1) and torch.equal(st, st1)
    # same GEMM without the MX outputs: identical bf16 y and aux
    z2 = torch.empty_like(z)
    y2 = F8.linear_fwd_mx(x, w, b, act="relu", aux=z2, drop_p=0.1, drop_seed=3)
    assert torch.equal(y, y2) and torch.equal(z, z2)
    # skip-C: the MX copies are the same, the consumer's forward uses them
    F8.clear_saved()
    y3 = F8.linear_fwd_mx(x, w, b, act="relu", aux=z2, drop_p=0.1, drop_seed=3, mx_out=True, mx_skip_c=True)
    (q3, s3), (qt3, st3) = F8.cached_dual(y3)
    torch.cuda.synchronize()
    assert torch.equal(q3, q1) and torch.equal(qt3, qt1) and torch.equal(s3, s1) and torch.equal(st3, st1)
    if K % 128 == 0 and N % 128 == 0:
        w2 = (torch.randn(K, N, generator=g) * 0.05).to(torch.bfloat16).cuda()
        out_skip = F8.linear_fwd_mx(y3, w2, save=True)
        F8.clear_saved()
        out_ref = F8.linear_fwd_mx(y, w2, save=True)
        torch.cuda.synchronize()
        assert torch.equal(out_skip, out_ref)
    F8.clear_saved()
    # dgrad with relu' + dropout: MX(dx) from the epilogue == dual quantization of dx
    if N % 128 == 0:
        dy = torch.randn(M, N, generator=g).to(torch.bfloat16).cuda()
        dx = F8.linear_dgrad_mx(dy, w, dact_src=z, dact="relu", drop_p=0.1, drop_seed=4, mx_out=True)
        (dq, ds_), (dqt, dst) = F8.cached_dual(dx)
        (dq1, ds1), (dqt1, dst1) = F8.mx_quantize_dual(dx)
        dx_plain = F8.linear_dgrad_mx(dy, w, dact_src=z, dact="relu", drop_p=0.1, drop_seed=4)
        torch.cuda.synchronize()
        assert torch.equal(dx, dx_plain)
        assert torch.equal(dq, dq1) and torch.equal(ds_, ds1) and torch.equal(dqt, dqt1) and torch.equal(dst, dst1)
    F8.clear_saved()


@pytest.mark.parametrize("M,W", [(256, 1024), (96, 768), (8192, 1024)])
def test_layernorm_mx_outputs_equal_dual_quantizer(M, W):
    """layernorm_fwd_mx: y, mean, rstd identical to the plain LayerNorm kernel, and its MX row /
    column blocks identical to mx_quantize_dual(y); with skip_y the MX copies are unchanged."""
    from tensorflow_k8s_amd.ops import transformer as T
    g = torch.Generator().manual_seed(W)
    x = (torch.randn(M, W, generator=g) * 3).to(torch.bfloat16).cuda()
    gm = (torch.rand(W, generator=g) + 0.5).cuda()
    bt = (torch.randn(W, generator=g) * 0.1).cuda()
    F8.clear_saved()
    y0, mu0, rs0 = T.layernorm_fwd(x, gm, bt, 1e-6)
    y1, mu1, rs1 = T.layernorm_fwd(x, gm, bt, 1e-6, mx_out=True)
    (q, s), (qt, st) = F8.cached_dual(y1)
    (q0, s0), (qt0, st0) = F8.mx_quantize_dual(y0)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1) and torch.equal(mu0, mu1) and torch.equal(rs0, rs1)
    assert torch.equal(q, q0) and torch.equal(s, s0) and torch.equal(qt, qt0) and torch.equal(st, st0)
    y2, _, _ = T.layernorm_fwd(x, gm, bt, 1e-6, mx_out=True, skip_y=True)
    (q2, s2), (qt2, st2) = F8.cached_dual(y2)
    torch.cuda.synchronize()
    assert torch.equal(q2, q0) and torch.equal(qt2, qt0) and torch.equal(s2, s0) and torch.equal(st2, st0)
    F8.clear_saved()


@pytest.mark.parametrize("M,W,drop", [(256, 1024, 0.1), (96, 768, 0.0), (8192, 1024, 0.3)])
def test_layernorm_bwd_mx_outputs(M, W, drop):
    """layernorm_bwd mx_out: dx / dropout(dx) identical to the plain kernel, dgamma / dbeta / consumer
    bias gradient equal up to the f32 summation order (rows are blocked differently), and the MX row /
    column blocks identical to mx_quantize_dual of the consumer gradient."""
    from tensorflow_k8s_amd.ops import transformer as T
    g = torch.Generator().manual_seed(M + W)
    x = (torch.randn(M, W, generator=g) * 2).to(torch.bfloat16).cuda()
    dy = torch.randn(M, W, generator=g).to(torch.bfloat16).cuda()
    dres = torch.randn(M, W, generator=g).to(torch.bfloat16).cuda()
    gm = (torch.rand(W, generator=g) + 0.5).cuda()
    bt = torch.zeros(W).cuda()
    _, mu, rs = T.layernorm_fwd(x, gm, bt, 1e-6)
    outs = {}
    from tensorflow_k8s_amd.ops._lib import lib
    lib().ln_bwd_set_fast(0)  # the plain side of the comparison on the generic kernel the MX mode extends
    for mx in (False, True):
        F8.clear_saved()
        dg, db, dbias = torch.zeros(W).cuda(), torch.zeros(W).cuda(), torch.zeros(W).cuda()
        r = T.layernorm_bwd(dy, x, gm, mu, rs, dg, db, dres=dres, accumulate=True,
                            drop=(drop, 7) if drop > 0 else None, dbias=dbias, mx_out=mx)
        cons = r[1] if drop > 0 else r
        outs[mx] = (r, dg, db, dbias, F8.cached_dual(cons) if mx else None, cons)
    torch.cuda.synchronize()
    lib().ln_bwd_set_fast(1)
    (r0, dg0, db0, bs0, _, c0), (r1, dg1, db1, bs1, mxq, c1) = outs[False], outs[True]
    assert torch.equal(c0, c1)
    for a, b in ((dg0, dg1), (db0, db1), (bs0, bs1)):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-3)
    (q, s), (qt, st) = mxq
    (q1, s1), (qt1, st1) = F8.mx_quantize_dual(c1)
    torch.cuda.synchronize()
    assert torch.equal(q, q1) and torch.equal(s, s1) and torch.equal(qt, qt1) and torch.equal(st, st1)
    F8.clear_saved()


def test_fp8_dgrad_column_sums_and_mx_only_output():
    """MX-fp8 dgrad with the fused column sums and mx_skip_c: the sums equal those of the bf16 dx a
    storing call produces, and the MX copies are the same bytes either way."""
    from tensorflow_k8s_amd.ops import gemm as G
    M, N, K = 1024, 512, 256
    g = torch.Generator().manual_seed(11)
    dy = (torch.randn(M, N, generator=g) * 0.5).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).cuda()
    mask = G.relu_mask_pack(torch.randn(M, K, generator=g)).cuda()
    try:
        cs1 = torch.zeros(K, device="cuda")
        dx = F8.linear_dgrad_mx(dy, w, dact_src=mask, dact="relu", drop_p=0.1, drop_seed=2, mx_out=True, colsum=cs1)
        q1 = [t.clone() for pair in F8.cached_dual(dx) for t in pair]
        cs2 = torch.zeros(K, device="cuda")
        dx2 = F8.linear_dgrad_mx(dy, w, dact_src=mask, dact="relu", drop_p=0.1, drop_seed=2, mx_out=True,
                                 colsum=cs2, mx_skip_c=True)
        q2 = [t.clone() for pair in F8.cached_dual(dx2) for t in pair]
        torch.cuda.synchronize()
        ref = dx.float().sum(0)
        tol = 1e-3 * float(ref.abs().max()) + 1e-4
        assert float((cs1 - ref).abs().max()) <= tol and float((cs2 - ref).abs().max()) <= tol
        assert all(torch.equal(a, b) for a, b in zip(q1, q2))
        with pytest.raises(RuntimeError):
            F8._check_stored(dx2)  # no bf16 values behind an mx_skip_c output
    finally:
        F8.clear_saved()
