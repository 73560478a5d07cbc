"""Halo-tile 3x3 weight gradient (csrc/kernels/conv_hwgrad.hip) vs the fp32 PyTorch reference
(torch.nn.grad.conv2d_weight on the CPU) and vs the im2col gather it replaces, on every band shape
it serves: ResNet 3x3 convs at stride 1 (56/28/14/7 outputs) and stride 2 (28/14), input and
output channel counts that differ, and partial multi-image bands (N not a multiple of NB).
Reference behaviour: SURVEY §2.4 K4 (conv weight gradient)."""
import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G

pytestmark = pytest.mark.gpu

# (N, H, C, K, stride)
SHAPES = [(2, 56, 64, 64, 1), (2, 28, 128, 128, 1), (2, 14, 64, 128, 1), (4, 7, 128, 64, 1),
          (2, 56, 64, 128, 2), (2, 28, 128, 64, 2)]


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("N,H,C,K,st", SHAPES)
def test_hwgrad_matches_fp32(N, H, C, K, st):
    g = G.ConvGeom(N, H, H, C, K, 3, 3, st, st, 1, 1)
    assert G.hwgrad_slabs(g) > 0, "shape must be served by the halo weight gradient"
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C).to(torch.bfloat16)
    dy = torch.randn(N, g.P, g.Q, K).to(torch.bfloat16)
    ref = torch.zeros(K, 3, 3, C)
    G.conv_wgrad(dy, x, g, ref)  # CPU branch: fp32 torch.nn.grad.conv2d_weight
    gw = torch.full((K, 3, 3, C), float("nan"), device="cuda")
    G.conv_wgrad(dy.cuda(), x.cuda(), g, gw)
    # accumulate onto an existing gradient as well
    gw2 = torch.ones(K, 3, 3, C, device="cuda")
    G.conv_wgrad(dy.cuda(), x.cuda(), g, gw2, accumulate=True)
    # the im2col gather path on the same inputs
    G.HWGRAD = False
    try:
        gg = torch.zeros(K, 3, 3, C, device="cuda")
        G.conv_wgrad(dy.cuda(), x.cuda(), g, gg)
    finally:
        G.HWGRAD = True
    torch.cuda.synchronize()
    assert torch.isfinite(gw).all()
    assert _rel(gw.cpu(), ref) < 2e-3, _rel(gw.cpu(), ref)
    assert _rel(gw2.cpu() - 1.0, ref) < 2e-3
    assert _rel(gw.cpu(), gg.cpu()) < 2e-3


@pytest.mark.parametrize("N", [2, 3])
def test_stem_wgrad_matches_fp32(N):
    """ResNet conv1 (7x7/s2/p3, RGB padded to 8 channels): the direct stem kernel computes channels
    0..3 and stores zeros for the padding channels 4..7."""
    g = G.ConvGeom(N, 224, 224, 8, 64, 7, 7, 2, 2, 3, 3)
    assert G.stem_wgrad_slabs(g, 3) > 0
    torch.manual_seed(1)
    x = torch.zeros(N, 224, 224, 8)
    x[..., :3] = torch.randn(N, 224, 224, 3)
    x = x.to(torch.bfloat16)
    dy = torch.randn(N, 112, 112, 64).to(torch.bfloat16)
    ref = torch.zeros(64, 7, 7, 8)
    G.conv_wgrad(dy, x, g, ref)
    gw = torch.full((64, 7, 7, 8), float("nan"), device="cuda")
    G.conv_wgrad(dy.cuda(), x.cuda(), g, gw, cin_used=3)
    gg = torch.zeros(64, 7, 7, 8, device="cuda")
    G.conv_wgrad(dy.cuda(), x.cuda(), g, gg)  # cin_used unknown -> im2col gather path
    torch.cuda.synchronize()
    gw = gw.cpu()
    assert torch.isfinite(gw).all()
    assert float(gw[..., 3:].abs().max()) == 0.0
    assert _rel(gw, ref) < 2e-3, _rel(gw, ref)
    assert _rel(gw, gg.cpu()) < 2e-3


@pytest.mark.parametrize("N", [2, 3])
def test_stem_fwd_matches_fp32(N):
    """ResNet conv1 forward on the direct halo kernel: output and BN batch statistics vs the fp32
    CPU reference and vs the implicit-GEMM gather."""
    g = G.ConvGeom(N, 224, 224, 8, 64, 7, 7, 2, 2, 3, 3)
    torch.manual_seed(2)
    x = torch.zeros(N, 224, 224, 8)
    x[..., :3] = torch.randn(N, 224, 224, 3)
    x = x.to(torch.bfloat16)
    w = torch.zeros(64, 7, 7, 8)
    w[..., :3] = torch.randn(64, 7, 7, 3) * 0.1
    w = w.to(torch.bfloat16)
    st_ref = torch.zeros(2 * 64)
    y_ref = G.conv_fwd(x, w, g, stats=st_ref, shards=1)
    assert G.stem_fwd_ok(g, 3)
    st = torch.zeros(16 * 2 * 64, device="cuda")
    y = G.conv_fwd(x.cuda(), w.cuda(), g, stats=st, shards=16, cin_used=3)
    st2 = torch.zeros(16 * 2 * 64, device="cuda")
    y2 = G.conv_fwd(x.cuda(), w.cuda(), g, stats=st2, shards=16)  # gather path
    torch.cuda.synchronize()
    assert _rel(y.cpu().float(), y_ref.float()) < 1e-2
    assert _rel(y.cpu().float(), y2.cpu().float()) < 1e-2
    s = st.view(16, 2, 64).sum(0).cpu()
    assert _rel(s[0], st_ref.view(2, 64)[0]) < 1e-3 and _rel(s[1], st_ref.view(2, 64)[1]) < 1e-3
