"""CPU tier: the executor's hand-written ResNet backward (incl. the fused BN-reduce plumbing and
mask-from-y) against torch autograd on the same arena weights."""
import torch
import torch.nn.functional as F

from reference_models import _bn, resnet_loss
from tensorflow_k8s_amd.models.resnet import Bottleneck, ResNet, synthetic_imagenet
from tensorflow_k8s_amd.runtime.arena import ParamArena


class _Round(torch.autograd.Function):
    """Emulates bf16 storage of activations and of their gradients (what the executor keeps)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def _block_case(cin, width, stride, prev_tail=False):
    torch.manual_seed(0)
    a = ParamArena()
    b = Bottleneck(a, 2, 0, cin, width, stride)
    a.finalize("cpu")
    with torch.no_grad():
        for bn in b.bns():
            bn.gamma.master.uniform_(0.5, 1.5)
            bn.beta.master.uniform_(-0.2, 0.2)
    x = torch.randn(4, 16, 16, cin).relu().to(torch.bfloat16)
    out = b.forward(x)
    dout = torch.randn(out.shape).to(torch.bfloat16)
    dx = b.backward(dout)
    rd = _Round.apply
    L = {p.name: p.master.clone().requires_grad_(True) for p in a.params}
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)

    def conv(l, h):
        return rd(F.conv2d(h, L[l.w.name].to(torch.bfloat16).float().permute(0, 3, 1, 2), stride=l.stride, padding=l.pad))

    def bn(l, h):
        return _bn(h, L[l.gamma.name], L[l.beta.name], l.eps)

    o = rd(F.relu(bn(b.bn1, conv(b.conv1, xr))))
    o = rd(F.relu(bn(b.bn2, conv(b.conv2, o))))
    o = bn(b.bn3, conv(b.conv3, o))
    sc = bn(b.bn_sc, conv(b.conv_sc, xr)) if b.proj else xr
    r = rd(F.relu(o + sc))
    (r * dout.float().permute(0, 3, 1, 2)).sum().backward()
    assert float((r.permute(0, 2, 3, 1) - out.float()).norm() / r.norm()) < 1e-2
    assert float((xr.grad.permute(0, 2, 3, 1) - dx.float()).norm() / xr.grad.norm()) < 0.1
    for p in a.params:
        ref = L[p.name].grad
        assert float((p.grad - ref).norm() / (ref.norm() + 1e-12)) < 0.15, p.name


def test_bottleneck_identity():
    _block_case(256, 64, 1)


def test_bottleneck_projection_strided():
    _block_case(256, 128, 2)


def test_resnet_gradients_track_autograd():
    # shallow (one bottleneck per stage): full-depth random-init ResNets are chaotic enough that two
    # bf16 runs with different summation orders decorrelate (measured), which says nothing about
    # the backward implementation; the per-block tests above cover every block type at depth 1.
    torch.manual_seed(0)
    m = ResNet(50, num_classes=10, stages=[1, 1, 1, 1]).to("cpu")
    with torch.no_grad():  # non-zero residual branches so every layer gets gradient
        for bn in m.batchnorms():
            bn.gamma.master.fill_(1.0)
    m.arena.refresh_compute()
    x, y = synthetic_imagenet(8, "cpu", image_size=96, num_classes=10)
    loss, _ = m.forward_backward(x, y)
    rl, leaves = resnet_loss(m, x, y, m.label_smoothing, emulate_bf16=True)
    rl.backward()
    assert abs(float(loss.mean()) - float(rl)) < 0.05
    g = torch.cat([p.grad.reshape(-1) for p in m.arena.params])
    r = torch.cat([leaves[p.name].grad.reshape(-1) for p in m.arena.params])
    cos = float(F.cosine_similarity(g, r, dim=0))
    assert cos > 0.9, cos


def test_relu_bitmask_pack_roundtrip_and_backward():
    """Packed relu mask (bit e of byte i = a[8i+e] > 0): round trip, and the BN backward driven by
    the bitmask equals the one driven by the bf16 activation (the ResNet tail saves the mask only)."""
    import torch
    from tensorflow_k8s_amd.ops import norm as BN
    g = torch.Generator().manual_seed(0)
    C, M = 16, 40
    y = torch.randn(M, C, generator=g).to(torch.bfloat16)
    r = torch.randn(M, C, generator=g).to(torch.bfloat16)
    st = BN.BNState(C, "cpu")
    BN.bn_stats(y, st)
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    BN.bn_finalize(st, M, gamma, beta, 1e-5, 0.1, None, None)
    a, mk = BN.bn_apply(y, st, True, r=r, mask=True)
    assert mk.dtype == torch.uint8 and mk.numel() == M * C // 8
    assert torch.equal(BN.unpack_relu_mask(mk, a.shape), a.float() > 0)
    da = torch.randn(M, C, generator=g).to(torch.bfloat16)
    res = []
    for m in (a, mk):
        dg, db = torch.zeros(C), torch.zeros(C)
        dy, _, dres = BN.bn_backward(da, m, y, st, gamma, dg, db, M, want_dres=True)
        res.append((dy, dres, dg, db))
    for u, v in zip(*res):
        assert torch.equal(u, v)


def test_bn_pool_states_and_deferred_finalize_cpu():
    """ResNet.to() puts every BN layer's accumulators in one BNPool buffer (zeroed once per training
    step when the fused finalize kernels are on); on the CPU a deferred finalize runs at once (the
    fused kernels are GPU-only), so the executor's numbers are unchanged."""
    import torch
    from tensorflow_k8s_amd.models.resnet import ResNet, synthetic_imagenet
    from tensorflow_k8s_amd.ops import norm as BN
    m = ResNet(50, num_classes=10, stages=[1, 1, 1, 1]).to("cpu")
    pool = m._bn_pool
    bns = m.batchnorms()
    assert len(pool.states) == len(bns) and all(bn.st is st for bn, st in zip(bns, pool.states))
    assert all(st.pooled and st.stats.data_ptr() >= pool.buf.data_ptr() for st in pool.states)
    x, y = synthetic_imagenet(2, "cpu", image_size=64, num_classes=10)
    loss, _ = m.forward_backward(x, y)
    assert torch.isfinite(loss).all()
    assert all(float(st.stats.abs().sum()) == 0.0 for st in pool.states)  # every finalize re-zeroed its shards
    st = BN.BNState(8, "cpu")
    BN.bn_finalize(st, 4.0, torch.ones(8), torch.zeros(8), 1e-5, 0.1, None, None, defer=True)
    assert st.fin is None  # not pooled / not on the GPU: finalized immediately
