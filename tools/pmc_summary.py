#!/usr/bin/env python3
"""Summarise a rocprofv3 PMC database (rocpd SQLite): per kernel (name filter), mean counter
values per dispatch and mean duration.   python tools/pmc_summary.py DB [name-substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    pats = sys.argv[2:]
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for d, k, n, v, du in rows:
        if pats and not any(p in k for p in pats):
            continue
        key = k[:90]
        per[key][n].append(v)
        dur[key][d] = du
    for k, cs in per.items():
        ds = list(dur[k].values())
        print(f"== {k}  dispatches={len(ds)} mean_ns={sum(ds) / len(ds):.0f}")
        for n, vs in sorted(cs.items()):
            print(f"   {n:32s} {sum(vs) / len(vs) * len(vs) / len(ds):.4g}")


if __name__ == "__main__":
    main()
