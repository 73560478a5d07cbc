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
