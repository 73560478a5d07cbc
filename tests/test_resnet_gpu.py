"""ResNet-50 end-to-end on the GPU executor vs the same executor on CPU (fp32 reference ops),
plus hipGraph capture/replay equivalence."""
import pytest
import torch

from tensorflow_k8s_amd.models.resnet import ResNet, synthetic_imagenet
from tensorflow_k8s_amd.runtime.optimizer import SGD
from tensorflow_k8s_amd.runtime.trainer import StepRunner

pytestmark = pytest.mark.gpu


def test_resnet50_step_matches_cpu():
    torch.manual_seed(0)
    mc = ResNet(50, num_classes=100).to("cpu")
    mg = ResNet(50, num_classes=100).to("cuda")
    mg.arena.master.copy_(mc.arena.master)
    mg.arena.refresh_compute()
    x, y = synthetic_imagenet(8, "cpu", image_size=128, num_classes=100)
    lc, _ = mc.forward_backward(x, y)
    lg, _ = mg.forward_backward(x.cuda(), y.cuda())
    assert abs(float(lc.mean()) - float(lg.mean())) < 0.05
    gc, gg = mc.arena.grad, mg.arena.grad.cpu()
    cos = float(torch.nn.functional.cosine_similarity(gc, gg, dim=0))
    assert cos > 0.9, cos


def test_hipgraph_replay_matches_eager():
    torch.manual_seed(0)
    ms = [ResNet(50, num_classes=10).to("cuda") for _ in range(2)]
    ms[1].arena.master.copy_(ms[0].arena.master)
    ms[1].arena.refresh_compute()
    x, y = synthetic_imagenet(16, "cuda", image_size=96, num_classes=10)
    runs = []
    for m, graph in zip(ms, (False, True)):
        opt = SGD(m.arena, lr=0.01)
        r = StepRunner(m, opt, None, (x, y), use_graph=graph)
        for _ in range(4):
            r.step()
        torch.cuda.synchronize()
        runs.append((r.last_loss(), m.arena.master.clone()))
    assert abs(runs[0][0] - runs[1][0]) < 1e-2
    assert float((runs[0][1] - runs[1][1]).norm() / runs[0][1].norm()) < 1e-2


@pytest.mark.parametrize("mode", ["1", "auto"])
def test_side_stream_wgrad_matches_single_stream(mode, monkeypatch):
    """Weight gradients on the side HIP stream (runtime/streams.py), eager (mode "1") and
    hipGraph-captured ("auto"): the same training trajectory as the single-stream step."""
    from tensorflow_k8s_amd.runtime import streams
    torch.manual_seed(0)
    ms = [ResNet(50, num_classes=10).to("cuda") for _ in range(2)]
    ms[1].arena.master.copy_(ms[0].arena.master)
    ms[1].arena.refresh_compute()
    x, y = synthetic_imagenet(16, "cuda", image_size=96, num_classes=10)
    runs = []
    for m, smode in zip(ms, ("0", mode)):
        monkeypatch.setattr(streams, "MODE", smode)
        opt = SGD(m.arena, lr=0.01)
        r = StepRunner(m, opt, None, (x, y), use_graph=mode == "auto")
        for _ in range(4):
            r.step()
        torch.cuda.synchronize()
        runs.append((r.last_loss(), m.arena.master.clone()))
    assert abs(runs[0][0] - runs[1][0]) < 1e-2
    assert float((runs[0][1] - runs[1][1]).norm() / runs[0][1].norm()) < 1e-2


def test_bn_finalize_in_apply_resnet_step_matches(monkeypatch):
    """A captured ResNet-50 training step with the BN finalizes folded into the BN passes (pooled
    accumulators zeroed once per step, ops/norm.py FUSED_FIN) follows the separate-finalize step:
    loss, master weights and the BN running statistics after 4 SGD steps."""
    from tensorflow_k8s_amd.ops import norm as BN
    torch.manual_seed(0)
    ms = [ResNet(50, num_classes=10).to("cuda") for _ in range(2)]
    ms[1].arena.master.copy_(ms[0].arena.master)
    ms[1].arena.refresh_compute()
    x, y = synthetic_imagenet(16, "cuda", image_size=96, num_classes=10)
    runs = []
    for m, fused in zip(ms, (False, True)):
        monkeypatch.setattr(BN, "FUSED_FIN", fused)
        opt = SGD(m.arena, lr=0.01)
        r = StepRunner(m, opt, None, (x, y), use_graph=True)
        for _ in range(4):
            r.step()
        torch.cuda.synchronize()
        runs.append((r.last_loss(), m.arena.master.clone(), torch.cat([b.tensor.reshape(-1) for b in m.arena.buffers])))
    assert abs(runs[0][0] - runs[1][0]) < 1e-3 * abs(runs[0][0]), (runs[0][0], runs[1][0])
    assert float((runs[0][1] - runs[1][1]).norm() / runs[0][1].norm()) < 1e-3
    assert float((runs[0][2] - runs[1][2]).norm() / runs[0][2].norm()) < 1e-3
