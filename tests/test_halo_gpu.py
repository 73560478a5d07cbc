"""Halo-tile direct 3x3 convolution (csrc/kernels/conv_halo.hip) vs the fp32 CPU reference and vs
the implicit-GEMM gather it replaces, on ResNet stage-1/2 shapes (56x56x64, 28x28x128): forward
with the fused BN batch statistics, and the stride-1 dgrad (run as a forward conv over dY) with the
fused BN-backward reduction and the premasked dz store. Reference behaviour: SURVEY §2.4 K2/K3."""
import pytest
import torch

from tensorflow_k8s_amd.ops import gemm as G
from tensorflow_k8s_amd.ops import norm as BN
from tensorflow_k8s_amd.ops._lib import lib

pytestmark = pytest.mark.gpu

SHAPES = [(2, 56, 64), (3, 56, 64), (2, 28, 128)]


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("N,HW,C", SHAPES)
def test_halo_forward_with_stats(N, HW, C):
    g = G.ConvGeom(N, HW, HW, C, C, 3, 3, 1, 1, 1, 1)
    level = 2 if C == 128 else 1  # stage-2 shapes are opt-in (TFK_HALO=2)
    torch.manual_seed(0)
    x = torch.randn(N, HW, HW, C).to(torch.bfloat16)
    w = (torch.randn(C, 3, 3, C) * 0.05).to(torch.bfloat16)
    st_ref = torch.zeros(2 * C)
    y_ref = G.conv_fwd(x, w, g, stats=st_ref, shards=1)
    out = {}
    for halo in (1, 0):
        lib().halo_set(level if halo else 0)
        try:
            st = torch.zeros(16 * 2 * C, device="cuda")
            y = G.conv_fwd(x.cuda(), w.cuda(), g, stats=st, shards=16)
            torch.cuda.synchronize()
        finally:
            lib().halo_set(-1)
        out[halo] = (y.cpu(), st.view(16, 2, C).sum(0).cpu())
    yh, sh = out[1]
    assert _rel(yh.float(), y_ref.float()) < 1e-2
    assert _rel(sh, st_ref.view(2, C)) < 1e-3
    yg, sg = out[0]
    assert _rel(yh.float(), yg.float()) < 5e-3 and _rel(sh, sg) < 1e-3


@pytest.mark.parametrize("N,HW,C", SHAPES)
@pytest.mark.parametrize("premask", [False, True])
def test_halo_dgrad_with_bn_reduce(N, HW, C, premask):
    g = G.ConvGeom(N, HW, HW, C, C, 3, 3, 1, 1, 1, 1)
    level = 2 if C == 128 else 1
    assert G.dgrad_as_fwd_geom(g) is not None
    torch.manual_seed(1)
    dy = torch.randn(N, HW, HW, C).to(torch.bfloat16)
    w = (torch.randn(C, 3, 3, C) * 0.05).to(torch.bfloat16)
    y = torch.randn(N, HW, HW, C).to(torch.bfloat16)

    def spec(dev):
        st = BN.BNState(C, dev)
        st.mean.copy_(torch.linspace(-0.1, 0.1, C)); st.invstd.copy_(torch.linspace(0.8, 1.2, C))
        st.scale.copy_(torch.linspace(0.5, 1.5, C)); st.shift.copy_(torch.linspace(-0.2, 0.2, C))
        return BN.BNReduce(y.to(dev), st, premask=premask)

    ref = spec("cpu")
    dx_ref = G.conv_dgrad(dy, w, g, bnr=ref)
    res = {}
    for halo in (1, 0):
        lib().halo_set(level if halo else 0)
        try:
            b = spec("cuda")
            dx = G.conv_dgrad(dy.cuda(), w.cuda(), g, bnr=b)
            torch.cuda.synchronize()
        finally:
            lib().halo_set(-1)
        res[halo] = (dx.cpu(), b.st.sums.view(b.st.shards, 3, C).sum(0).cpu())
    dxh, sh = res[1]
    assert _rel(dxh.float(), dx_ref.float()) < 1e-2
    sref = ref.st.sums.view(1, 3, C)[0]
    assert _rel(sh[:2], sref[:2]) < 2e-3
    dxg, sg = res[0]
    assert _rel(dxh.float(), dxg.float()) < 5e-3
