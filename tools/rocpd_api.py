#!/usr/bin/env python3
"""Host API calls in a rocprofv3 database (``--hip-trace`` / ``--runtime-trace`` runs): count, total
and max duration per API name, plus the durations of the last N calls of one API (e.g.
``hipGraphLaunch``: is the host's graph submission on the critical path of a replayed step?).

    python tools/rocpd_api.py rn_results.db [--api hipGraphLaunch] [--last 12]
"""
from __future__ import annotations

import argparse
import sqlite3


def _cols(c, name):
    return [r[1] for r in c.execute(f"pragma table_info('{name}')").fetchall()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--api", default="hipGraphLaunch")
    ap.add_argument("--last", type=int, default=12)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    objs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')").fetchall()]
    # the API-region view: has start / end / name columns and is not the kernel view
    src = None
    for o in objs:
        cols = _cols(c, o)
        if {"start", "end", "name"} <= set(cols) and o.lower() in ("regions", "region", "regions_and_samples"):
            src = o
            break
    if src is None:
        for o in objs:
            cols = _cols(c, o)
            if {"start", "end", "name"} <= set(cols) and "kernel" not in o.lower():
                src = o
                break
    if src is None:
        print("no region table with start/end/name; objects:", objs)
        return
    print(f"source: {src}")
    rows = c.execute(f"select name, count(*), sum(end - start), max(end - start) from {src} "
                     f"group by name order by sum(end - start) desc limit 25").fetchall()
    print("api                                   calls     total ms      max us")
    for n, k, t, m in rows:
        print(f"{str(n)[:36]:36s} {k:7d} {t / 1e6:12.3f} {m / 1e3:11.1f}")
    last = c.execute(f"select start, end from {src} where name like ? order by start desc limit ?",
                     (f"%{a.api}%", a.last)).fetchall()
    if last:
        last = last[::-1]
        print(f"last {len(last)} {a.api}: duration us, interval to the next call us")
        for i, (s, e) in enumerate(last):
            nxt = (last[i + 1][0] - s) / 1e3 if i + 1 < len(last) else float("nan")
            print(f"  {(e - s) / 1e3:10.1f}  {nxt:10.1f}")


if __name__ == "__main__":
    main()
