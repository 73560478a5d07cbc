#!/usr/bin/env python3
"""Per-op kernel times of one eager training step, with a roofline column per op.

Every native entry point is bracketed by device events (TFK_OPPROF, ops/_lib.py); for each call
the tool prints its time, FLOP rate, the bytes its tensor arguments span, and the floor
max(flops / PEAK, bytes / BW) -> eff = floor / time. GEMM calls are labelled with their operand
modes, tile and split count, so a rocprofv3 per-kernel total can be broken down per layer.

    python tools/op_profile.py --model resnet50 --batch 256 [--steps 2] [--out gpurun_out/op.jsonl]
    python tools/op_profile.py ... --ab-persist 1     # A/B the persistent GEMM grid in one process
"""
import argparse
import collections
import json
import os
import sys

os.environ.setdefault("TFK_OPPROF", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

PEAK = 2.3e15   # achievable dense bf16 MFMA FLOP/s (guide: 2.5 PF spec)
BW = 6.0e12     # achievable HBM B/s (guide: 6.3 TB/s measured)
AMODES = {0: "kin", 1: "kout", 2: "cfwd", 3: "cdgrad"}
BMODES = {0: "kin", 1: "kout", 2: "cwgrad"}
EPIS = {0: "bf16", 1: "f32"}


def _tensors(x):
    if isinstance(x, dict) and "shape" in x:
        yield x
    elif isinstance(x, list):
        for y in x:
            yield from _tensors(y)


def _bytes(args) -> int:
    tot = 0
    for t in _tensors(args):
        n = 1
        for d in t["shape"]:
            n *= d
        tot += n * t["esize"]
    return tot


def describe(rec):
    """(label, flops, bytes) of one profiled call."""
    op, a = rec["op"], rec["args"]
    if op == "gemm":
        M, N, K = a[3], a[4], a[5]
        amode, bmode, epi, bm, bn = a[9], a[10], a[11], a[12], a[13]
        splits, batch, conv = a[21], a[22], a[27]
        bnr = a[28]
        geo = ""
        if amode in (2, 3) or bmode == 2:
            geo = f" {conv[7]}x{conv[8]}/s{conv[9]} C{conv[3]}->{conv[6]} {conv[1]}x{conv[2]}"
        tag = f"gemm {AMODES[amode]}.{BMODES[bmode]}.{EPIS[epi]}{'+bnr' if bnr else ''} t{bm}x{bn} s{splits}"
        label = f"{tag} M{M} N{N} K{K}{geo}"
        # A operand of a conv gather is the whole activation; tensors passed cover everything touched
        return label, 2.0 * M * N * K * batch, _bytes(a), tag
    if op == "gemm_mxfp8":
        M, N, K = a[5], a[6], a[7]
        f32 = a[4].get("esize") == 4 if isinstance(a[4], dict) else False
        tag = f"mxfp8 {'wgrad.f32' if f32 else 'bf16'}"
        # the fp8 MFMA peak is twice bf16's: count half the FLOPs against PEAK
        return f"{tag} M{M} N{N} K{K}", 2.0 * M * N * K / 2, _bytes(a[:5]), tag
    return op, 0.0, _bytes(a), op


def summarize(recs, top: int = 60, file=sys.stdout):
    tot = sum(r["ms"] for r in recs)
    rows = []
    for r in recs:
        label, fl, by, tag = describe(r)
        floor = max(fl / PEAK, by / BW) * 1e3
        rows.append((r["ms"], label, fl, by, floor, tag))
    print(f"# {len(recs)} native calls, {tot:.3f} ms of kernel time (events)", file=file)
    by_tag = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for ms, _, _, _, floor, tag in rows:
        by_tag[tag][0] += ms
        by_tag[tag][1] += floor
        by_tag[tag][2] += 1
    print(f"{'ms':>8s} {'floor':>8s} {'eff':>5s} {'calls':>5s}  op", file=file)
    for tag, (ms, fl, n) in sorted(by_tag.items(), key=lambda kv: -kv[1][0]):
        print(f"{ms:8.3f} {fl:8.3f} {100 * fl / max(ms, 1e-9):4.0f}% {n:5d}  {tag}", file=file)
    print(f"\n# top {top} calls", file=file)
    print(f"{'ms':>8s} {'TF/s':>7s} {'GB/s':>7s} {'eff':>5s}  call", file=file)
    for ms, label, fl, by, floor, _ in sorted(rows, key=lambda x: -x[0])[:top]:
        s = ms / 1e3
        print(f"{ms:8.3f} {fl / s / 1e12:7.1f} {by / s / 1e9:7.0f} {100 * floor / max(ms, 1e-9):4.0f}%  {label}", file=file)
    floor_tot = sum(x[4] for x in rows)
    print(f"\n# sum of floors {floor_tot:.3f} ms vs {tot:.3f} ms measured ({100 * floor_tot / max(tot, 1e-9):.0f}%)",
          file=file)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--out", default="")
    ap.add_argument("--top", type=int, default=60)
    ap.add_argument("--ab-persist", type=int, default=0, help="also profile with the persistent GEMM grid off")
    ap.add_argument("--fp8", type=int, default=0, help="transformer models: MX-fp8 linear GEMMs")
    args = ap.parse_args()

    from tensorflow_k8s_amd.models import build_model, synthetic_batch
    from tensorflow_k8s_amd.ops._lib import lib
    from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
    from tensorflow_k8s_amd.runtime.optimizer import SGD, AdamW
    from tensorflow_k8s_amd.runtime.trainer import StepRunner

    dev = torch.device("cuda", 0)
    model = build_model(args.model, **({"fp8": True} if args.fp8 else {})).to(dev)
    opt = SGD(model.arena, lr=0.1, momentum=0.9) if args.model.startswith(("resnet", "lenet")) else \
        AdamW(model.arena, lr=1e-4)
    strat = MultiWorkerMirroredStrategy(model.arena)
    strat.configure_optimizer(opt)
    runner = StepRunner(model, opt, strat, synthetic_batch(model, args.batch, dev, seed=1), use_graph=False)
    L = lib()
    variants = [("persist", 1)] + ([("no-persist", 0)] if args.ab_persist else [])
    out = open(args.out, "w") if args.out else None
    for _ in range(args.warmup):
        runner.step()
    L.records()
    for name, flag in variants:
        if hasattr(L._mod, "gemm_set_persist"):
            L._mod.gemm_set_persist(flag)
        runner.step()
        L.records()
        recs = []
        for _ in range(args.steps):
            runner.step()
            recs = L.records()  # keep the last step
        print(f"\n########## {args.model} bs{args.batch} [{name}]")
        summarize(recs, args.top)
        if out:
            for r in recs:
                out.write(json.dumps({"variant": name, **r}) + "\n")
    if out:
        out.close()


if __name__ == "__main__":
    main()
