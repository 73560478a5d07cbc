"""Halo-tile 3x3 weight gradient (csrc/kernels/conv_hwgrad.hip) vs the fp32 PyTorch reference
(torch.nn.grad.conv2d_weight on the CPU) and vs the im2col gather it replaces, on every band shape
it serves: ResNet 3x3 convs at stride 1 (56/28/14/7 outputs) and stride 2 (28/14/7), input and
output channel counts that differ, and partial multi-image bands (N not a multiple of NB).
Reference behaviour: SURVEY §2.4 K4 (conv weight gradient)."""
import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G

pytestmark = pytest.mark.gpu

# (N, H, C, K, stride)
SHAPES = [(2, 56, 64, 64, 1), (2, 28, 128, 128, 1), (2, 14, 64, 128, 1), (4, 7, 128, 64, 1),
          (2, 56, 64, 128, 2), (2, 28, 128, 64, 2), (3, 14, 64, 64, 2)]


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
