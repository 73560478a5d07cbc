#!/usr/bin/env python3
"""Join rocprofv3 PMC passes (one rocpd SQLite database per counter group, e.g. tools/pmc_resnet.sh)
per kernel and print derived per-kernel ratios, heaviest kernels first:

  wait%     SQ_WAIT_ANY / SQ_WAVE_CYCLES          share of wave-cycles waiting on anything
  ldsw%     SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES     share of wave-cycles waiting on LDS results
  conf%     SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  mfma%     SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs x CUs x 4 SIMDs)   MFMA pipe busy
            share (the MFMA counter sums SIMD-cycles chip-wide, GRBM_GUI_ACTIVE sums the 8 XCDs'
            clocks: a 16x16x32 bf16 MFMA counts 16 busy cycles and 32 BF16 MOPs)
  bfTF/s    SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 flops over the kernel time
  rd/wr     FETCH_SIZE / WRITE_SIZE (KiB) over the kernel time, GB/s

Counters are summed over every dispatch of a kernel name before dividing (time-weighted).
    python tools/pmc_derived.py gpurun_out/pmc_r50 [--top 25] [--cus 256] [--steps 2]"""
import argparse
import glob
import os
import sqlite3
from collections import defaultdict


def load(root):
    cnt = defaultdict(lambda: defaultdict(float))  # kernel -> counter -> sum
    dur = defaultdict(dict)                          # kernel -> {(db, dispatch): ns}
    for db in sorted(glob.glob(os.path.join(root, "**", "*.db"), recursive=True)):
        c = sqlite3.connect(db)
        try:
            rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration "
                             "from counters_collection").fetchall()
        except sqlite3.Error:
            continue
        for d, k, n, v, du in rows:
            cnt[k][n] += v
            dur[k][(db, d)] = du
    return cnt, dur


def short(k: str) -> str:
    k = k.replace("(anonymous namespace)::", "").replace("tfk::", "")
    return k.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=1, help="training steps in each pass (calls / us per step)")
    a = ap.parse_args()
    cnt, dur = load(a.root)
    rows = []
    for k, cs in cnt.items():
        by_db = defaultdict(list)
        for (db, _), ns in dur[k].items():
            by_db[db].append(ns)
        # one pass's dispatches = one step's worth: time from the pass with the most dispatches
        ns_list = max(by_db.values(), key=len)
        rows.append((sum(ns_list), len(ns_list), k, cs))
    rows.sort(key=lambda r: -r[0])

    def ratio(cs, a_, b_, scale=100.0):
        return f"{scale * cs[a_] / cs[b_]:.0f}" if cs.get(b_) else "-"

    print(f"{'kernel':60s} {'calls':>5s} {'us':>8s} {'wait%':>5s} {'ldsw%':>5s} {'conf%':>5s} "
          f"{'mfma%':>5s} {'bfTF/s':>6s} {'rdGB/s':>7s} {'wrGB/s':>7s}")
    for tot, n, k, cs in rows[:a.top]:
        n, step_us = n // a.steps, tot / 1e3 / a.steps
        mf = "-"
        if cs.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            mf = f"{100.0 * cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (cs['GRBM_GUI_ACTIVE'] / a.xcds * a.cus * 4):.1f}"
        tf = f"{cs['SQ_INSTS_VALU_MFMA_MOPS_BF16'] * 512 / tot / 1e3:.0f}" if cs.get("SQ_INSTS_VALU_MFMA_MOPS_BF16") else "-"
        # the FETCH/WRITE passes time their own dispatches: divide by this pass-independent total
        rd = f"{cs['FETCH_SIZE'] * 1024 / tot:.0f}" if "FETCH_SIZE" in cs and tot else "-"
        wr = f"{cs['WRITE_SIZE'] * 1024 / tot:.0f}" if "WRITE_SIZE" in cs and tot else "-"
        print(f"{short(k):60s} {n:5d} {step_us:8.1f} {ratio(cs, 'SQ_WAIT_ANY', 'SQ_WAVE_CYCLES'):>5s} "
              f"{ratio(cs, 'SQ_WAIT_INST_LDS', 'SQ_WAVE_CYCLES'):>5s} "
              f"{ratio(cs, 'SQ_LDS_BANK_CONFLICT', 'SQ_ACTIVE_INST_LDS'):>5s} {mf:>5s} {tf:>6s} {rd:>7s} {wr:>7s}")


if __name__ == "__main__":
    main()
