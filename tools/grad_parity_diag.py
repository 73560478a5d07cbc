#!/usr/bin/env python3
"""Per-parameter gradient agreement of the gfx950 ResNet executor with the CPU fp32 executor,
printed in backward order (loss-side first), for a few (image size, batch, residual gamma) configs:
shows where GPU/CPU gradient cosine degrades and whether it tracks BN batch size (cancellation in
the bf16 BN backward) or depth.

    python tools/grad_parity_diag.py [--configs 64:8:0.5,128:16:0.5,64:8:0.05]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="64:8:0.5,128:16:0.5,64:8:0.05")
    ap.add_argument("--stages", default="1,1,1,1")
    ap.add_argument("--perturb", type=float, default=0.0,
                    help="instead of the GPU, compare the CPU (fp32) run with a CPU run on weights perturbed by this "
                         "relative amount (bf16 rounding is ~4e-3): measures the network's own sensitivity")
    args = ap.parse_args()
    from tensorflow_k8s_amd.models.resnet import ResNet, synthetic_imagenet
    stages = [int(s) for s in args.stages.split(",")]
    for cfg in args.configs.split(","):
        size, bs, gam = int(cfg.split(":")[0]), int(cfg.split(":")[1]), float(cfg.split(":")[2])
        grads, losses = {}, {}
        runs = (("cpu", "cpu", 0.0), ("cuda", "cuda", 0.0)) if not args.perturb else (("cpu", "cpu", 0.0),
                                                                                       ("cuda", "cpu", args.perturb))
        for key, dev, eps in runs:
            m = ResNet(50, stages=stages, num_classes=100).to(dev, seed=3)
            for p in m.arena.params:
                if p.name.endswith("/gamma") and float(p.master.abs().sum()) == 0.0:
                    p.master.fill_(gam)
            if eps:
                g = torch.Generator().manual_seed(1)
                m.arena.master.mul_(1 + eps * torch.randn(m.arena.master.shape, generator=g).to(m.arena.master.device))
            m.arena.refresh_compute()
            x, y = synthetic_imagenet(bs, "cpu", image_size=size, num_classes=100, seed=5)
            loss, _ = m.forward_backward(x.to(dev), y.to(dev))
            losses[key] = float(loss.float().mean())
            grads[key] = [(p.name, p.grad.detach().float().cpu().clone()) for p in sorted(m.arena.params, key=lambda p: p.offset)]
        rows = [(n, round(cos(g, dict(grads["cpu"])[n]), 5), round(float(dict(grads["cpu"])[n].norm()), 6))
                for n, g in grads["cuda"]]
        print(json.dumps({"config": cfg, "loss_cpu": losses["cpu"], "loss_gpu": losses["cuda"],
                          "min_cos": min(r[1] for r in rows if r[2] > 0)}), flush=True)
        for r in rows:
            print(f"   {r[1]:8.5f}  |g|={r[2]:.3e}  {r[0]}")


if __name__ == "__main__":
    main()
