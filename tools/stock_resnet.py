#!/usr/bin/env python3
"""Stock PyTorch-ROCm comparator for BASELINE.md: ResNet-50 v1.5 written with torch.nn (MIOpen
convs / BN, hipBLASLt FC), channels_last, bf16 autocast, SGD momentum, synthetic data, eager.
This is what a user would get WITHOUT tfk's kernels/executor on the same MI355X.

    python tools/stock_resnet.py --batch 256 --steps 20 --warmup 5 [--compile 0]
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.c1, self.b1 = nn.Conv2d(cin, width, 1, bias=False), nn.BatchNorm2d(width)
        self.c2, self.b2 = nn.Conv2d(width, width, 3, stride, 1, bias=False), nn.BatchNorm2d(width)
        self.c3, self.b3 = nn.Conv2d(width, cout, 1, bias=False), nn.BatchNorm2d(cout)
        self.sc = None
        if stride != 1 or cin != cout:
            self.sc = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        o = self.relu(self.b1(self.c1(x)))
        o = self.relu(self.b2(self.c2(o)))
        o = self.b3(self.c3(o))
        return self.relu(o + (self.sc(x) if self.sc is not None else x))


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for si, n in enumerate([3, 4, 6, 3]):
            w = 64 * 2 ** si
            for bi in range(n):
                layers.append(Bottleneck(cin, w, 2 if bi == 0 and si > 0 else 1))
                cin = w * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(self.layers(self.stem(x)), 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--compile", type=int, default=0)
    ap.add_argument("--precision", default="autocast", choices=["autocast", "bf16"],
                    help="autocast: f32 weights under bf16 autocast; bf16: bf16 weights + activations")
    ap.add_argument("--fused", type=int, default=1, help="fused (single-kernel) SGD")
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = ResNet50().to(dev).to(memory_format=torch.channels_last)
    if a.precision == "bf16":
        m = m.to(torch.bfloat16)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, **({"fused": True} if a.fused else {}))
    crit = nn.CrossEntropyLoss(label_smoothing=0.1)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    if a.precision == "bf16":
        x = x.to(torch.bfloat16)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    fwd = torch.compile(m) if a.compile else m

    def step():
        opt.zero_grad(set_to_none=True)
        if a.precision == "autocast":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = crit(fwd(x), y)
        else:
            loss = crit(fwd(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"comparator": f"stock_pytorch_{a.precision}" + ("_fusedsgd" if a.fused else "") +
                      ("_compile" if a.compile else ""), "batch": a.batch,
                      "ms_per_step": round(dt * 1000, 3), "img_s": round(a.batch / dt, 2),
                      "loss": float(loss)}))


if __name__ == "__main__":
    main()
