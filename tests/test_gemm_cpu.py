

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
