#!/usr/bin/env python3
"""Host (enqueue) time vs device time of eager training steps: is the eager step launch-bound?

    python tools/host_overhead.py [--model resnet50] [--batch 256] [--steps 10] [--profile 0|1]

Prints the host time to enqueue K steps (no synchronisation inside) and the wall time once the
device has drained. host ~= wall means the host cannot keep the GPU fed (the multi-GPU steps run
eagerly). --profile 1: cProfile of the enqueue loop, top functions by cumulative time.
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.models import build_model, synthetic_batch  # noqa: E402
from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy  # noqa: E402
from tensorflow_k8s_amd.runtime.optimizer import SGD  # noqa: E402
from tensorflow_k8s_amd.runtime.trainer import StepRunner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--profile", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = build_model(a.model).to(dev)
    opt = SGD(m.arena, lr=0.01, momentum=0.9)
    strat = MultiWorkerMirroredStrategy(m.arena)
    r = StepRunner(m, opt, strat, synthetic_batch(m, a.batch, dev, seed=1), use_graph=False)
    for _ in range(3):
        r.step()
    torch.cuda.synchronize()
    prof = cProfile.Profile() if a.profile else None
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    for _ in range(a.steps):
        r.step()
    if prof:
        prof.disable()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    print(f"{a.model} bs{a.batch} eager: host enqueue {t_host / a.steps * 1e3:.2f} ms/step, "
          f"wall {t_wall / a.steps * 1e3:.2f} ms/step")
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
