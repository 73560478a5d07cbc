

def test_lib_gemm_shape_classes(monkeypatch):
    """Plain-GEMM routing to hipBLASLt covers only the measured shape classes (ops.gemm.LIB_GEMM)."""
    from tensorflow_k8s_amd.ops import gemm as G
    assert G.lib_gemm_ok("fwd", 8192, 33728, 1024) and G.lib_gemm_ok("fwd", 8192, 3072, 1024)
    assert not G.lib_gemm_ok("fwd", 8192, 1024, 1024) and not G.lib_gemm_ok("fwd", 256, 33728, 1024)
    assert G.lib_gemm_ok("dgrad", 8192, 1024, 33728) and not G.lib_gemm_ok("dgrad", 2048, 1024, 3072)
    assert G.lib_gemm_ok("wgrad", 33728, 1024, 8192)
    assert not G.lib_gemm_ok("wgrad", 4096, 1024, 8192) and not G.lib_gemm_ok("wgrad", 256, 64, 802816)
    monkeypatch.setattr(G, "LIB_GEMM", False)
    assert not G.lib_gemm_ok("fwd", 8192, 33728, 1024)


def test_relu_mask_reference_matches_bf16_preactivation():
    """uint8 relu-mask aux (1 bit per pre-activation) gives the same activation backward as the
    bf16 pre-activation copy (CPU reference path of ops.gemm)."""
    import torch
    from tensorflow_k8s_amd.ops import gemm as G
    g = torch.Generator().manual_seed(0)
    M, N, K = 37, 48, 32
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, generator=g).to(torch.bfloat16)
    z = torch.empty(M, N, dtype=torch.bfloat16)
    m = torch.empty(M, N // 8, dtype=torch.uint8)
    y1 = G.linear_fwd(x, w, act="relu", aux=z)
    y2 = G.linear_fwd(x, w, act="relu", aux=m)
    assert torch.equal(y1, y2)
    assert torch.equal(G.relu_mask_unpack(m), (z.float() > 0).float())
    assert torch.equal(G.relu_mask_pack(z.float()), m)
    dy = torch.randn(M, K, generator=g).to(torch.bfloat16)
    w2 = torch.randn(K, N, generator=g).to(torch.bfloat16)
    assert torch.equal(G.linear_dgrad(dy, w2, dact_src=z, dact="relu"), G.linear_dgrad(dy, w2, dact_src=m, dact="relu"))


def test_dgrad_colsum_reference_is_bias_gradient_of_consumer():
    """linear_dgrad(colsum=g) adds the column sums of the returned dx (before any residual) to g --
    the bias gradient of the layer consuming dx (CPU reference path)."""
    import torch
    from tensorflow_k8s_amd.ops import gemm as G
    g = torch.Generator().manual_seed(2)
    M, N, K = 24, 16, 40
    dy = torch.randn(M, N, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, generator=g).to(torch.bfloat16)
    z = torch.randn(M, K, generator=g)
    m = G.relu_mask_pack(z)
    cs = torch.full((K,), 2.0)
    dx = G.linear_dgrad(dy, w, dact_src=m, dact="relu", colsum=cs)
    assert torch.allclose(cs, dx.float().sum(0) + 2.0, atol=1e-5)
    assert torch.equal(dx, G.linear_dgrad(dy, w, dact_src=m, dact="relu"))
