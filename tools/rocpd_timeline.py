#!/usr/bin/env python3
"""Timeline view of a rocprofv3 ``--kernel-trace`` database: how much of a training step the GPU is
idle (no kernel on any queue), which kernel boundaries the idle time sits at, and -- per hardware
queue -- how long the MAIN queue (the input-gradient chain) waits while side queues (weight
gradients on the side streams, comm) still run.

    python tools/rocpd_timeline.py rn_results.db --steps 13 [--last 3] [--top 25] [--first stem_fwd]

Step windows: with ``--first SUBSTR`` a step starts at every dispatch of a kernel whose name contains
SUBSTR (the model's first kernel: ``stem_fwd``, ``embed_fwd``) and the last ``--last`` complete
steps are taken; without it the dispatches are split evenly by count (a captured step replays the
same kernel sequence, but anything outside the steps -- the final loss read-back -- shifts that split).
Prints busy / idle time per step, the overlap factor (sum of kernel time / busy time: > 1 when side
streams run concurrently), per-queue busy time, the largest all-idle gaps, and the largest gaps of
the main queue with what the other queues ran meanwhile.
"""
from __future__ import annotations

import argparse
import collections
import sqlite3


def _busy(iv):
    tot, cur = 0, None
    for s, e in sorted(iv):
        if cur is None or s > cur:
            tot += e - s
            cur = e
        elif e > cur:
            tot += e - cur
            cur = e
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, required=True, help="training steps the trace covers (warmup included)")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--first", default=None, help="substring of the first kernel of a step")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select start, end, name, queue_id from kernels order by start").fetchall()
    if a.first:
        starts = [i for i, r in enumerate(rows) if a.first in r[2]]
        k = max(1, round(len(starts) / a.steps))  # e.g. encoder + decoder embeddings: 2 per step
        starts = starts[len(starts) % k::k] if len(starts) % k else starts[::k]
        if len(starts) < a.last + 1:
            raise SystemExit(f"fewer than {a.last + 1} dispatches of '{a.first}'")
        b0, b1 = starts[-a.last - 1], starts[-1]
        win = rows[b0:b1]
    else:
        per = len(rows) // a.steps
        win = rows[-per * a.last:]
    nsteps = a.last
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
    print(f"window: last {nsteps} steps, {len(win) // nsteps} dispatches/step"
          + (f" (aligned on '{a.first}')" if a.first else ""))
    print(f"per step: span {span / 1e6 / nsteps:.3f} ms, busy {busy / 1e6 / nsteps:.3f} ms, "
          f"idle {idle / 1e6 / nsteps:.3f} ms ({100 * idle / span:.1f}%), kernel sum {ksum / 1e6 / nsteps:.3f} ms "
          f"(overlap x{ksum / max(busy, 1):.2f}), {len(gaps) / nsteps:.0f} gaps/step")
    # per hardware queue: dispatches and busy time (a captured step's parallel branches -- the
    # weight-gradient side streams, the comm stream -- land on their own queues)
    per_q = collections.defaultdict(list)
    for s_, e_, name, q in win:
        per_q[q].append((s_, e_, name))
    print("per queue (per step): dispatches, busy ms")
    for q, iv in sorted(per_q.items(), key=lambda kv: -len(kv[1])):
        print(f"  queue {q}: {len(iv) / nsteps:6.0f}  {_busy([(s, e) for s, e, _ in iv]) / 1e6 / nsteps:8.3f}")
    by_pair = collections.Counter()
    for g, p, n in gaps:
        by_pair[(p[:60], n[:60])] += g
    print("largest all-idle time by (previous kernel -> next kernel), per step:")
    for (p, n), g in by_pair.most_common(a.top):
        print(f"  {g / 1e3 / nsteps:8.1f} us   {p}  ->  {n}")
    # the largest single idle gaps, located by step and offset from the step's first dispatch (a
    # gap that moves from step to step points at the host: graph-node submission falling behind)
    if a.first:
        step_t0 = [rows[i][0] for i in starts[-a.last - 1:]]
        singles = []
        cur, prev = None, None
        for s, e, name, q in win:
            if cur is not None and s > cur:
                k = max(i for i, t in enumerate(step_t0) if t <= s)
                singles.append((s - cur, k, (cur - step_t0[k]) / 1e3, prev, name))
            if cur is None or e > cur:
                cur, prev = e, name
        print("largest single idle gaps: us, step, offset into the step (us), previous -> next")
        for g, k, off, p, n in sorted(singles, reverse=True)[:10]:
            print(f"  {g / 1e3:8.1f}  {k}  {off:9.1f}   {p[:50]}  ->  {n[:50]}")
    # main queue = the one with the most dispatches; its gaps = time the chain waits (on an event of
    # another queue, or a launch). Attribute each gap to what the other queues ran inside it. (A
    # replayed hipGraph may move a stream's chain between hardware queues after a fork / join: read
    # this section only when the other queues' kernels are side-stream kernels.)
    mq = max(per_q, key=lambda q: len(per_q[q]))
    mk = sorted(per_q[mq])
    others = sorted((s, e, n) for q, iv in per_q.items() if q != mq for s, e, n in iv)
    mgaps = collections.Counter()
    inside = collections.Counter()
    total = 0
    for (s0, e0, n0), (s1, e1, n1) in zip(mk, mk[1:]):
        g = s1 - e0
        if g <= 2000:  # < 2 us: a launch boundary, not a wait
            continue
        total += g
        mgaps[(n0[:55], n1[:55])] += g
        for s, e, n in others:
            if e <= e0 or s >= s1:
                continue
            inside[n[:70]] += min(e, s1) - max(s, e0)
    print(f"main queue {mq}: waits > 2 us total {total / 1e6 / nsteps:.3f} ms per step; largest by "
          f"(previous -> next main-queue kernel):")
    for (p, n), g in mgaps.most_common(a.top):
        print(f"  {g / 1e3 / nsteps:8.1f} us   {p}  ->  {n}")
    print("other queues' kernel time inside those waits, per step:")
    for n, g in inside.most_common(a.top):
        print(f"  {g / 1e3 / nsteps:8.1f} us   {n}")


if __name__ == "__main__":
    main()
