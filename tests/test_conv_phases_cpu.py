"""CPU check of the sub-pixel (phase) decomposition behind the strided-conv dgrad
(ops.gemm._phases): every output phase of conv_transpose equals a stride-1 correlation of dY
with the phase's tap subset, exactly as the per-phase A_CONV_DGRAD GEMM computes it."""
import pytest
import torch
import torch.nn.functional as F

from tensorflow_k8s_amd.ops import gemm as G


def _phase_dgrad(dy, wt, g, a, b, Ha, Wb, r0, s0, Rp, Sp, php, pwp):
    # dx_phase[n,i,j,c] = sum_{r',s',co} dY[n, i+php-r', j+pwp-s', co] * wt[c, r0+sh*r', s0+sw*s', co]
    N, P, Q, K = dy.shape
    out = torch.zeros(N, Ha, Wb, wt.shape[0], dtype=torch.float64)
    for rr in range(Rp):
        for ss in range(Sp):
            wk = wt[:, r0 + g.sh * rr, s0 + g.sw * ss, :].double()  # [C][K]
            for i in range(Ha):
                pi = i + php - rr
                if not 0 <= pi < P:
                    continue
                for j in range(Wb):
                    qj = j + pwp - ss
                    if 0 <= qj < Q:
                        out[:, i, j, :] += dy[:, pi, qj, :].double() @ wk.t()
    return out


@pytest.mark.parametrize("cfg", [(2, 8, 8, 4, 6, 3, 3, 2, 1), (1, 7, 9, 3, 5, 3, 3, 2, 1), (1, 9, 9, 2, 3, 5, 5, 3, 2),
                                 (2, 6, 6, 4, 4, 2, 2, 2, 0)])
def test_phase_decomposition_matches_conv_transpose(cfg):
    N, H, W, C, K, R, S, st, pd = cfg
    g = G.ConvGeom(N, H, W, C, K, R, S, st, st, pd, pd)
    torch.manual_seed(0)
    dy = torch.randn(N, g.P, g.Q, K, dtype=torch.float64)
    w = torch.randn(K, R, S, C, dtype=torch.float64)
    out_pad = (g.H - ((g.P - 1) * g.sh - 2 * g.ph + R), g.W - ((g.Q - 1) * g.sw - 2 * g.pw + S))
    ref = F.conv_transpose2d(dy.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), stride=st, padding=pd,
                             output_padding=out_pad).permute(0, 2, 3, 1)
    wt = w.permute(3, 1, 2, 0)  # [C][R][S][K] = conv_weight_t layout
    phases = G._phases(g)
    assert phases is not None
    covered = torch.zeros(H, W, dtype=torch.int32)
    for ph in phases:
        a, b = ph[0], ph[1]
        got = _phase_dgrad(dy, wt, g, *ph)
        assert torch.allclose(got, ref[:, a::st, b::st, :], atol=1e-9), ph
        covered[a::st, b::st] += 1
    assert bool((covered == 1).all())


def test_pointwise_strided_has_empty_phases():
    assert G._phases(G.ConvGeom(1, 8, 8, 4, 4, 1, 1, 2, 2, 0, 0)) is None
