

def test_no_vendor_gemm_in_the_op_layer():
    """Every GEMM of the model path runs on the framework's HIP kernels: the op layer has no library
    routing left (round 4 sent plain GEMMs of some shape classes to hipBLASLt through aten)."""
    import inspect
    from tensorflow_k8s_amd.ops import gemm as G
    src = inspect.getsource(G)
    assert not hasattr(G, "lib_gemm_ok") and not hasattr(G, "LIB_GEMM")
    for call in ("torch.mm(", "torch.matmul(", "aten.mm", "aten.addmm", "F.linear("):
        assert call not in src, call


def test_lds_dma_only_through_the_asm_helper():
    """Every LDS-DMA in the kernel library goes through common.h's lds_dma (inline asm): with the
    builtin, hipcc puts s_waitcnt vmcnt(0) before each later ds_read_b64_tr_b16, so the K-outer GEMMs
    and the weight-gradient kernels wait for the next stage's DMA mid-tile (profiles/perf_log_r5.md),
    and a builtin next to the helper could be handed a stale compiler-tracked M0."""
    import glob
    import os
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "kernels")
    srcs = glob.glob(os.path.join(root, "*.hip")) + glob.glob(os.path.join(root, "*.h"))
    assert srcs
    for path in srcs:
        with open(path) as f:
            text = f.read()
        for builtin in ("__builtin_amdgcn_raw_ptr_buffer_load_lds", "__builtin_amdgcn_raw_buffer_load_lds",
                        "__builtin_amdgcn_global_load_lds"):
            assert builtin not in text, (os.path.basename(path), builtin)
    with open(os.path.join(root, "common.h")) as f:
        assert "offen lds" in f.read()


def test_dgrad_splitk_policy():
    """Plain input gradients with too few 256x256 output tiles and a long reduction (the tied-logits
    dgrad) take the split-K path; wide outputs and short reductions do not."""
    from tensorflow_k8s_amd.ops import gemm as G
    calls = []

    class FakeLib:
        def gemm_splits(self, K, s):
            return s

        def splitk_reduce(self, *a):
            calls.append("reduce")
    import torch
    orig_lib, orig_gemm, orig_ws = G.lib, G._gemm, G.workspace
    G.lib, G._gemm = (lambda: FakeLib()), (lambda *a, **k: calls.append(("gemm", k.get("splits"))))
    G.workspace = lambda dev, n, slot="": torch.empty(n)
    try:
        dx = torch.empty(8192, 1024, dtype=torch.bfloat16)
        assert G._dgrad_splitk(None, None, dx, 8192, 1024, 33728)  # 128 tiles, 33728-long reduction
        assert calls[0][0] == "gemm" and calls[0][1] >= 2 and calls[-1] == "reduce"
        assert not G._dgrad_splitk(None, None, torch.empty(8192, 4096, dtype=torch.bfloat16), 8192, 4096, 1024)
        assert not G._dgrad_splitk(None, None, dx, 8192, 1024, 1024)  # short reduction: one pass
        assert not G._dgrad_splitk(None, None, dx, 8192, 1024, 4096)  # FFN1's dgrad: unsplit 128x128
    finally:
        G.lib, G._gemm, G.workspace = orig_lib, orig_gemm, orig_ws


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


def test_wgrad_tail_split_policy():
    """The tied-embedding weight gradient (528 tiles = 2 rounds + 16) splits only its 16-tile tail;
    exact rounds, big tails and single-round gradients stay unsplit."""
    import torch
    from tensorflow_k8s_amd.ops import gemm as G
    calls = []

    class FakeLib:
        def gemm_splits(self, K, s):
            return s

        def splitk_reduce(self, *a):
            calls.append(("reduce", a[3]))
    orig = G.lib, G._gemm, G.workspace
    G.lib = lambda: FakeLib()
    G._gemm = lambda A, B, C, M, N, K, *a, **k: calls.append(("gemm", M, k.get("splits", 1)))
    G.workspace = lambda dev, n, slot="": torch.empty(n)
    try:
        gw = torch.empty(33728 * 1024)
        assert G._wgrad_tail_split(torch.empty(8192, 33728), None, gw, 33728, 1024, 8192, False)
        assert calls[0] == ("gemm", 32768, 1) and calls[1][1] == 960 and calls[1][2] >= 2
        assert calls[2] == ("reduce", 960 * 1024)
        assert not G._wgrad_tail_split(None, None, None, 4096, 4096, 8192, False)  # exactly 1 round
        assert not G._wgrad_tail_split(None, None, None, 4096, 1024, 8192, False)  # under a round
        n = len(calls)  # a row-tile wider than a round (K 76800 = 300 tiles, N 256): no 0-row launch
        assert not G._wgrad_tail_split(None, None, None, 256, 76800, 8192, False)
        assert len(calls) == n
    finally:
        G.lib, G._gemm, G.workspace = orig


def test_side_stream_wgrad_fill(monkeypatch):
    """Conv weight gradients issued on a side stream (runtime/streams.py sets ops._lib.ON_SIDE_STREAM)
    use 1/SIDE_WGRAD_FILL_DIV of the tuned split count and of the split-K fill target."""
    import torch
    from tensorflow_k8s_amd.ops import _lib
    from tensorflow_k8s_amd.ops import gemm as G
    seen = []
    monkeypatch.setattr(G, "on_gpu", lambda t: True)
    monkeypatch.setattr(G, "stem_wgrad_slabs", lambda g, c: 0)
    monkeypatch.setattr(G, "hwgrad_slabs", lambda g: 0)
    monkeypatch.setattr(G.tuning, "wgrad_config", lambda *a: ((256, 256), 16))
    monkeypatch.setattr(G, "_f32_out_splitk", lambda *a, **k: seen.append((k["force_splits"], k["split_target"])))
    g = G.ConvGeom(8, 14, 14, 256, 256, 1, 1, 1, 1, 0, 0)
    dy, x, gw = torch.empty(1), torch.empty(1), torch.empty(256 * 256)
    G.conv_wgrad(dy, x, g, gw)
    monkeypatch.setattr(_lib, "ON_SIDE_STREAM", True)
    G.conv_wgrad(dy, x, g, gw)
    d = G.SIDE_WGRAD_FILL_DIV
    assert seen == [(16, G.TARGET_BLOCKS), (max(1, 16 // d), G.TARGET_BLOCKS // d)]


def test_side_stream_linear_wgrad_fill(monkeypatch):
    """Linear weight gradients on a side stream halve the isolated-sweep fill; a layer's own
    split_target (set by the model from in-model measurements) is left alone."""
    import torch
    from tensorflow_k8s_amd.ops import _lib
    from tensorflow_k8s_amd.ops import gemm as G
    seen = []
    monkeypatch.setattr(G, "on_gpu", lambda t: True)
    monkeypatch.setattr(G.tuning, "wgrad_config", lambda *a: ((128, 128), 8))
    monkeypatch.setattr(G, "_f32_out_splitk", lambda *a, **k: seen.append((k["force_splits"], k["split_target"])))
    dy, x, gw = torch.empty(64, 1024), torch.empty(64, 1024), torch.empty(1024 * 1024)
    monkeypatch.setattr(_lib, "ON_SIDE_STREAM", True)
    G.linear_wgrad(dy, x, gw)
    G.linear_wgrad(dy, x, gw, split_target=512)
    d = G.SIDE_WGRAD_FILL_DIV
    assert seen[0] == (max(1, 8 // d), G.TARGET_BLOCKS // d)
    assert seen[1] == (None, 512)
