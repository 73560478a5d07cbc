"""Print per-step training loss of the tfk ResNet executor (debug/convergence check)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tensorflow_k8s_amd.models.resnet import ResNet, synthetic_imagenet
from tensorflow_k8s_amd.runtime.optimizer import SGD
from tensorflow_k8s_amd.runtime.trainer import StepRunner

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--lr", type=float, default=0.1)
ap.add_argument("--graph", type=int, default=0)
ap.add_argument("--device", default="cuda")
a = ap.parse_args()
m = ResNet(50).to(a.device)
opt = SGD(m.arena, lr=a.lr, momentum=0.9, weight_decay=5e-5)
x, y = synthetic_imagenet(a.batch, a.device)
r = StepRunner(m, opt, None, (x, y), use_graph=bool(a.graph))
for i in range(a.steps):
    r.step()
    print(i, round(r.last_loss(), 4), r.last_accuracy(), float(m.arena.grad.norm()), flush=True)
