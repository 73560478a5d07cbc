#!/usr/bin/env python3
"""Timeline view of a rocprofv3 ``--kernel-trace`` database: how much of a training step the GPU is
idle (no kernel on any queue), and which kernel boundaries the idle time sits at.

    python tools/rocpd_timeline.py gpurun_out/prof/rn/rn_results.db --steps 13 [--last 3] [--top 25]

The last ``--last`` steps of the trace are taken as the window (dispatches split evenly by count:
a captured step replays the same kernel sequence). Prints busy / idle time per step, the overlap
factor (sum of kernel time / busy time: > 1 when side streams run concurrently) and the largest
idle gaps with the kernels on either side -- launch-latency-bound chains of tiny kernels (BN
finalize, split-K reduce) show up here rather than in the per-kernel totals.
"""
from __future__ import annotations

import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, required=True, help="training steps the trace covers (warmup included)")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select start, end, name, queue_id from kernels order by start").fetchall()
    per = len(rows) // a.steps
    win = rows[-per * a.last:]
    t0, t1 = win[0][0], max(r[1] for r in win)
    busy, gaps, cur_end, prev = 0, [], None, None
    for s, e, name, q in win:
        if cur_end is None or s > cur_end:
            if cur_end is not None:
                gaps.append((s - cur_end, prev, name))
            busy += e - s
            cur_end = e
        else:
            if e > cur_end:
                busy += e - cur_end
                cur_end = e
        if cur_end == e:
            prev = name
    span = t1 - t0
    ksum = sum(e - s for s, e, _, _ in win)
    idle = span - busy
    print(f"window: last {a.last} steps, {per} dispatches/step")
    print(f"per step: span {span / 1e6 / a.last:.3f} ms, busy {busy / 1e6 / a.last:.3f} ms, "
          f"idle {idle / 1e6 / a.last:.3f} ms ({100 * idle / span:.1f}%), kernel sum {ksum / 1e6 / a.last:.3f} ms "
          f"(overlap x{ksum / max(busy, 1):.2f}), {len(gaps) / a.last:.0f} gaps/step")
    # per hardware queue: dispatches and busy time (a captured step's parallel branches -- the
    # weight-gradient side streams, the comm stream -- land on their own queues)
    per_q = collections.defaultdict(list)
    for s_, e_, _, q in win:
        per_q[q].append((s_, e_))
    print("per queue (per step): dispatches, busy ms")
    for q, iv in sorted(per_q.items(), key=lambda kv: -len(kv[1])):
        qb, qe = 0, None
        for s_, e_ in sorted(iv):
            if qe is None or s_ > qe:
                qb += e_ - s_
                qe = e_
            elif e_ > qe:
                qb += e_ - qe
                qe = e_
        print(f"  queue {q}: {len(iv) / a.last:6.0f}  {qb / 1e6 / a.last:8.3f}")
    by_pair = collections.Counter()
    for g, p, n in gaps:
        by_pair[(p[:60], n[:60])] += g
    print("largest idle time by (previous kernel -> next kernel), per step:")
    for (p, n), g in by_pair.most_common(a.top):
        print(f"  {g / 1e3 / a.last:8.1f} us   {p}  ->  {n}")


if __name__ == "__main__":
    main()
