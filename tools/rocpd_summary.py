#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 ``--kernel-trace`` SQLite database (rocpd schema, ROCm 7.x).

    python tools/rocpd_summary.py gpurun_out/prof/x_results.db --steps 13 [--csv out.csv] [--top 40]

Groups dispatches by kernel name: calls, total ms, ms per step, mean us, share of GPU time.
``--steps`` divides totals by the number of training steps the trace covers (warmup included).
"""
from __future__ import annotations

import argparse
import csv
import sqlite3


def summarize(db: str):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start) from kernels group by name").fetchall()
    rows.sort(key=lambda r: -r[2])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = summarize(a.db)
    tot = sum(r[2] for r in rows)
    print(f"GPU kernel time {tot / 1e6:.2f} ms total, {tot / 1e6 / a.steps:.3f} ms/step over {a.steps} steps")
    out = []
    for name, n, ns in rows:
        out.append({"kernel": name, "calls": n, "total_ms": round(ns / 1e6, 3),
                    "ms_per_step": round(ns / 1e6 / a.steps, 3), "avg_us": round(ns / 1e3 / n, 1),
                    "pct": round(100.0 * ns / tot, 2)})
    for r in out[:a.top]:
        print(f"{r['ms_per_step']:8.3f} ms/step {r['calls'] // a.steps:5d}/step {r['avg_us']:8.1f} us {r['pct']:5.1f}%  "
              f"{r['kernel'][:120]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
