#!/usr/bin/env python3
"""Tile sweep for every conv forward / dgrad GEMM a ResNet training step issues, timed with the
model's own epilogue (BN batch statistics on forwards, the fused BN-backward reduction + residual on
dgrads). The calls are discovered by recording one real ResNet step (ops.gemm.RECORD); each unique
(kind, geometry, epilogue flags) is then timed under every candidate tile (ops.gemm.FORCE_TILE),
interleaved rounds, median, against the analytic picker's choice (tuning off).

    python tools/conv_sweep.py [--model resnet50] [--batch 256] [--iters 10] [--rounds 3]
                               [--out gpurun_out/conv_sweep.jsonl] [--table tensorflow_k8s_amd/ops/tuned_conv.json]
"""
import argparse
import collections
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tensorflow_k8s_amd.ops import gemm as G  # noqa: E402
from tensorflow_k8s_amd.ops import norm as BN  # noqa: E402
from tensorflow_k8s_amd.ops import tuning  # noqa: E402

# (256, 128) / (128, 256): the 8-wave 3-stage g4 tiles (gemm_g4.hip NST = 3)
CANDS = {
    "fwd_pw": [(128, 128), (256, 256), (128, 64), (64, 128), (256, 64), (64, 64), (256, 128), (128, 256)],
    "fwd_gather": [(128, 128), (256, 256), (128, 64), (64, 128), (64, 64), (256, 64), (256, 128), (128, 256)],
    "dgrad_pw": [(128, 128), (256, 256), (128, 64), (64, 128), (256, 64), (64, 64), (256, 128), (128, 256)],
    "dgrad_fwd": [(128, 128), (256, 256), (128, 64), (64, 128), (64, 64), (256, 64), (256, 128), (128, 256)],
}


def bf(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def make_call(kind, geom, flags):
    g = G.ConvGeom(*[geom[i] for i in (0, 1, 2, 3, 6, 7, 8, 9, 10, 11, 12, 13, 14)])
    w = bf(g.K, g.R, g.S, g.C) * 0.05
    if kind == "fwd":
        x = bf(g.N, g.H, g.W, g.C)
        stats = torch.zeros(BN.SHARDS * 2 * g.K, device="cuda") if flags[0] else None
        return lambda: G.conv_fwd(x, w, g, stats, BN.SHARDS if flags[0] else 1)
    dy = bf(g.N, g.P, g.Q, g.K)
    has_resid, has_bnr, has_a, has_y2 = flags[0], flags[1], flags[2], flags[3]
    resid = bf(g.N, g.H, g.W, g.C) if has_resid else None
    spec = None
    if has_bnr:
        st = BN.BNState(g.C, "cuda")
        st.mean.uniform_(-0.1, 0.1)
        st.invstd.uniform_(0.5, 1.5)
        st2 = None
        if has_y2:
            st2 = BN.BNState(g.C, "cuda")
            st2.mean.uniform_(-0.1, 0.1)
            st2.invstd.uniform_(0.5, 1.5)
        spec = BN.BNReduce(bf(g.N, g.H, g.W, g.C), st, a=bf(g.N, g.H, g.W, g.C) if has_a else None,
                           y2=bf(g.N, g.H, g.W, g.C) if has_y2 else None, st2=st2)
    return lambda: G.conv_dgrad(dy, w, g, resid=resid, bnr=spec)


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--table", default="")
    args = ap.parse_args()
    tuning.ENABLED = False
    from tensorflow_k8s_amd.models import build_model, synthetic_batch
    m = build_model(args.model).to("cuda")
    batch = synthetic_batch(m, args.batch, "cuda", seed=1)
    G.RECORD = []
    m.forward_backward(*batch)
    torch.cuda.synchronize()
    calls = collections.Counter(G.RECORD)
    G.RECORD = None
    del m, batch
    torch.cuda.empty_cache()
    fh = open(args.out, "w") if args.out else None
    entries, saved = [], 0.0
    for (kind, geom, flags), count in sorted(calls.items(), key=lambda kv: kv[0][1]):
        if kind not in ("fwd", "dgrad_pw", "dgrad_fwd"):
            continue  # weight-gradient records belong to tools/wgrad_sweep.py
        pw = geom[7] == 1 and geom[8] == 1 and geom[9] == 1 and geom[10] == 1 and geom[11] == 0 and geom[12] == 0
        cands = CANDS["fwd_pw" if kind == "fwd" and pw else "fwd_gather" if kind == "fwd" else kind]
        fn = make_call(kind, geom, flags)
        G.FORCE_TILE = None
        res = {"default": []}
        res.update({t: [] for t in cands})
        ok = set(res)
        for _ in range(args.rounds):
            for t in list(res):
                if t not in ok:
                    continue
                G.FORCE_TILE = None if t == "default" else t
                try:
                    res[t].append(timeit(fn, args.iters))
                except RuntimeError:
                    ok.discard(t)
        G.FORCE_TILE = None
        med = {t: statistics.median(v) for t, v in res.items() if t in ok and v}
        best = min((t for t in med if t != "default"), key=med.get)
        gain = (med["default"] - med[best]) * count
        row = {"kind": kind, "geom": list(geom), "flags": list(flags), "count": count, "best": list(best),
               "best_us": round(med[best] * 1e6, 1), "default_us": round(med["default"] * 1e6, 1),
               "per_tile_us": {f"{t[0]}x{t[1]}": round(v * 1e6, 1) for t, v in med.items() if t != "default"}}
        print(json.dumps(row), flush=True)
        if fh:
            fh.write(json.dumps(row) + "\n")
            fh.flush()
        if med[best] < 0.97 * med["default"]:
            saved += gain
            entries.append({"kind": kind, "geom": list(geom), "tile": list(best), "us": row["best_us"],
                            "picker_us": row["default_us"]})
    print(json.dumps({"tuned_entries": len(entries), "est_saving_ms_per_step": round(saved * 1e3, 3)}), flush=True)
    if args.table:
        # several epilogue variants of one geometry: keep the entry with the largest total gain
        best_by_key = {}
        for e in entries:
            k = (e["kind"], tuple(e["geom"]))
            if k not in best_by_key or e["picker_us"] - e["us"] > best_by_key[k]["picker_us"] - best_by_key[k]["us"]:
                best_by_key[k] = e
        with open(args.table, "w") as f:
            json.dump({"source": f"tools/conv_sweep.py on MI355X ({args.model} bs{args.batch})",
                       "entries": list(best_by_key.values())}, f, indent=1)


if __name__ == "__main__":
    main()
