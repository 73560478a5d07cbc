#!/usr/bin/env python3
"""Tile x split-K sweep for the dense (1x1-conv) weight-gradient GEMMs of ResNet-50 at batch 256:
gw[Cout][Cin] (f32) = dY[pix][Cout]^T X[pix][Cin], K = pixels (12544 .. 802816). For every shape
it times each (tile, splits) candidate including the split-K slab reduce, and prints the winner
next to what ops.gemm.pick_tile chooses today. Interleaved rounds, median (one process).

    python tools/wgrad_sweep.py [--iters 20] [--rounds 3] [--out gpurun_out/wgrad_sweep.jsonl]
                                [--table tensorflow_k8s_amd/ops/tuned_wgrad.json]
--table writes the winners as the runtime's autotuning table (ops/tuning.py).
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops._lib import lib  # noqa: E402

# (Cout, Cin, pixels): ResNet-50 bs256 pointwise convs (conv1 Cin->w, conv3 w->4w, shortcut Cin->4w)
SHAPES = [(64, 64, 802816), (64, 256, 802816), (256, 64, 802816), (128, 256, 802816), (256, 256, 802816),
          (512, 256, 200704), (128, 512, 200704), (512, 128, 200704), (256, 512, 200704), (1024, 512, 50176),
          (256, 1024, 50176), (1024, 256, 50176), (512, 1024, 50176), (2048, 1024, 12544), (512, 2048, 12544),
          (2048, 512, 12544)]
TILES = [(64, 64), (128, 64), (64, 128), (128, 128), (64, 256), (256, 64), (256, 128), (128, 256), (256, 256)]
SPLITS = [1, 2, 4, 8, 16, 32, 64, 128, 256, 512]


def run_one(dy, x, gw, ws, M, N, K, tile, splits):
    ns = int(lib().gemm_splits(K, splits))
    stride = ((M * N + 3) // 4) * 4
    if ns == 1:
        G._gemm(dy, x, gw, M, N, K, M, N, N, G.A_KOUT, G.B_KOUT, G.EPI_F32, tile)
        return
    G._gemm(dy, x, ws, M, N, K, M, N, N, G.A_KOUT, G.B_KOUT, G.EPI_F32, tile, splits=splits, split_stride=stride)
    lib().splitk_reduce(ws, ns, stride, M * N, gw, None, False, 1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--table", default="", help="write the measured winners as ops/tuning.py's table")
    ap.add_argument("--models", default="", help="comma list (e.g. bert-base,transformer-big): sweep the dense "
                    "weight-gradient shapes one real step of each model issues instead of the ResNet list")
    ap.add_argument("--merge", action="store_true", help="merge into the existing --table instead of replacing it")
    args = ap.parse_args()
    shapes = SHAPES
    if args.models:
        from tensorflow_k8s_amd.models import build_model, synthetic_batch
        seen = []
        for name in args.models.split(","):
            m = build_model(name).to("cuda")
            bs = 256 if name.startswith("resnet") else {"bert-base": 64, "bert-large": 32}.get(name, 32)  # bench.py's
            b = synthetic_batch(m, bs, "cuda", seed=1)
            G.RECORD = []
            m.forward_backward(*b)
            torch.cuda.synchronize()
            for kind, shp, _ in G.RECORD:
                if kind == "wgrad" and shp not in seen and shp[0] % 8 == 0 and shp[1] % 8 == 0:
                    seen.append(shp)
            G.RECORD = None
            del m, b
            torch.cuda.empty_cache()
        shapes = seen
    from tensorflow_k8s_amd.ops import tuning
    tuning.ENABLED = False  # time the analytic picker's choice, not the table's
    fh = open(args.out, "w") if args.out else None
    dev = "cuda"
    ws = torch.empty(512 * 4096 * 1024 + 4096, device=dev)
    entries = []
    for M, N, K in shapes:
        dy = (torch.rand(K, M, device=dev) * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)
        gw = torch.empty(M, N, device=dev)
        ref = None
        cands = []
        for t in TILES:
            if t[0] > 2 * M or t[1] > 2 * N:
                continue
            for s in SPLITS:
                if int(lib().gemm_splits(K, s)) * M * N > ws.numel():
                    continue
                cands.append((t, s))
        times = {c: [] for c in cands}
        for _ in range(args.rounds):
            for c in cands:
                fn = lambda: run_one(dy, x, gw, ws, M, N, K, c[0], c[1])  # noqa: E731
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = (dy.float().t() @ x.float())
                t0 = time.perf_counter()
                for _ in range(args.iters):
                    fn()
                torch.cuda.synchronize()
                times[c].append((time.perf_counter() - t0) / args.iters)
        med = {c: statistics.median(v) for c, v in times.items()}
        best = min(med, key=med.get)
        run_one(dy, x, gw, ws, M, N, K, best[0], best[1])
        err = float((gw - ref).norm() / ref.norm())
        cur_t = G.pick_tile(M, N, splits_ok=True, big_ok=True, K=K, g4=True, rect_ok=True)
        tiles = ((M + cur_t[0] - 1) // cur_t[0]) * ((N + cur_t[1] - 1) // cur_t[1])
        cur_s = G.pick_splits(tiles, K)
        cur = min((c for c in med if c[0] == cur_t), key=lambda c: abs(c[1] - cur_s), default=None)
        row = {"M": M, "N": N, "K": K, "best_tile": best[0], "best_splits": best[1], "best_us": round(med[best] * 1e6, 1),
               "best_tflops": round(2 * M * N * K / med[best] / 1e12, 1), "picked": [cur_t, cur_s],
               "picked_us": round(med[cur] * 1e6, 1) if cur else None, "rel_err": err,
               "per_tile_best_us": {f"{t[0]}x{t[1]}": round(min(med[c] for c in med if c[0] == t) * 1e6, 1)
                                    for t in {c[0] for c in med}}}
        print(json.dumps(row), flush=True)
        if fh:
            fh.write(json.dumps(row) + "\n")
            fh.flush()
        entries.append({"M": M, "N": N, "K": K, "tile": list(best[0]), "splits": best[1], "us": row["best_us"],
                        "picker_us": row["picked_us"]})
    if args.table:
        if args.merge and os.path.exists(args.table):
            with open(args.table) as f:
                old = json.load(f)["entries"]
            keys = {(e["M"], e["N"], e["K"]) for e in entries}
            entries = [e for e in old if (e["M"], e["N"], e["K"]) not in keys] + entries
        with open(args.table, "w") as f:
            json.dump({"source": "tools/wgrad_sweep.py on MI355X", "entries": entries}, f, indent=1)


if __name__ == "__main__":
    main()
