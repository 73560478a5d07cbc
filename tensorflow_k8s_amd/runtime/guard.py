"""Guards for the first multi-GPU run: communicator self-test, hipGraph capture probe and unanimous
graph-or-eager agreement through the job store (SURVEY §5.3 failure detection; the failure modes
of k8s-operator.md:5 and the PS/WORKER task model of :6).

Why: the data-parallel step replays from ONE hipGraph that contains the RCCL bucket collectives.
RCCL calls made while a stream is capturing are recorded, not executed -- so if capture (or the
first replay) fails on one rank while the others succeed, the others block in their first replay
forever. Every decision that changes which collectives a rank will issue is therefore taken
unanimously, through the TCP store the communicators were bootstrapped from (not through RCCL,
which is the thing under test):

1. ``comm_self_test``: all-reduce of per-rank ramps (checked exactly against the closed form) and
   a broadcast of a pattern from rank 0, right after ``ncclCommInitRank``. Runs under the step
   watchdog (phase "comm self-test"); a mismatch raises ``CommSelfTestError`` (exit 143, the
   operator's retryable code) carrying the RCCL transport summary.
2. ``capture_probe``: capture fork -> all_reduce -> join into a tiny graph; every rank publishes
   ok / its error; only if ALL captured does every rank replay it twice and verify; a second
   agreement settles the result. Any failure anywhere -> every rank runs eager.
3. ``StepRunner`` (runtime/trainer.py) agrees again after capturing the real step, before its
   first replay; if any rank failed, all ranks drop their graphs and run the step eagerly
   in-process (no re-exec).

Fault injection (tests): ``TFK_FAULT_CAPTURE=probe|step|1`` (1 = probe) on
``TFK_FAULT_CAPTURE_RANK=<rank>|all`` (default all) raises inside the probe's / the step's capture.
"""
from __future__ import annotations

import datetime
import os
import time

import torch


class CommSelfTestError(RuntimeError):
    exit_code = 143  # retryable: the operator restarts the gang


class InjectedCaptureFault(RuntimeError):
    pass


def capture_fault(where: str, rank: int) -> None:
    """Raise InjectedCaptureFault when TFK_FAULT_CAPTURE names ``where`` for this rank."""
    v = os.environ.get("TFK_FAULT_CAPTURE", "")
    if not v or v == "0":
        return
    if (v if v != "1" else "probe") != where:
        return
    who = os.environ.get("TFK_FAULT_CAPTURE_RANK", "all")
    if who != "all" and int(who) != rank:
        return
    raise InjectedCaptureFault(f"injected {where} capture failure on rank {rank} (TFK_FAULT_CAPTURE={v})")


class Agreement:
    """Unanimous yes/no decisions among ``ranks`` (world ranks) through a key-value store
    (torch TCPStore / HashStore: set / wait / get). Each call of ``decide(name, ok, detail)``
    publishes this rank's vote under a fresh key and returns (all_ok, {rank: error} of the ranks
    that voted no). Without a store (single process) the local vote decides."""

    def __init__(self, store, rank: int, ranks, timeout_s: float = 300.0, prefix: str | None = None):
        self.store, self.rank, self.ranks = store, int(rank), sorted(int(r) for r in ranks)
        self.timeout_s = float(timeout_s)
        gen = os.environ.get("TFK_RESTART_GENERATION", "0") + "." + os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        self.prefix = prefix or f"tfk/agree/g{gen}"
        self._n: dict[str, int] = {}
        self.log: list[dict] = []

    def decide(self, name: str, ok: bool, detail: str = "") -> tuple[bool, dict]:
        n = self._n.get(name, 0)
        self._n[name] = n + 1
        if self.store is None or len(self.ranks) <= 1:
            bad = {} if ok else {self.rank: detail}
        else:
            base = f"{self.prefix}/{name}/{n}"
            self.store.set(f"{base}/{self.rank}", "ok" if ok else "err:" + (detail or "failed")[:600])
            keys = [f"{base}/{r}" for r in self.ranks]
            self.store.wait(keys, datetime.timedelta(seconds=self.timeout_s))
            bad = {}
            for r, k in zip(self.ranks, keys):
                v = bytes(self.store.get(k)).decode(errors="replace")
                if v != "ok":
                    bad[r] = v[4:] if v.startswith("err:") else v
        self.log.append({"decision": name, "ok": not bad, "failed_ranks": sorted(bad)})
        return not bad, bad

    @staticmethod
    def summary(bad: dict) -> str:
        return "; ".join(f"rank {r}: {e}" for r, e in sorted(bad.items()))


def _sync(dev: torch.device) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def comm_self_test(comm, n: int = 4096) -> dict:
    """All-reduce rank ramps + broadcast from rank 0 on ``comm``; exact checks. Returns timing and
    sizes; raises CommSelfTestError on a wrong result."""
    dev = comm.device
    w, r = comm.world, comm.rank
    t0 = time.perf_counter()
    base = torch.arange(n, dtype=torch.float32, device=dev)
    x = base + float(r)
    comm.all_reduce(x)
    # sum over ranks of (i + rank) = w*i + w(w-1)/2 -- small integers, exact in f32
    want = base * w + w * (w - 1) / 2.0
    pat = (torch.arange(n, dtype=torch.int32, device=dev) * 7 + 3) % 251
    b = pat.clone() if r == 0 else torch.zeros(n, dtype=torch.int32, device=dev)
    comm.broadcast(b, 0)
    _sync(dev)
    errs = []
    if not torch.equal(x, want):
        bad = int((x != want).sum())
        errs.append(f"all_reduce: {bad}/{n} wrong (first {x[(x != want).nonzero()[0]].tolist()})")
    if not torch.equal(b, pat):
        errs.append(f"broadcast: {int((b != pat).sum())}/{n} wrong")
    if errs:
        from ..parallel import comm as C
        raise CommSelfTestError(f"communicator self-test failed on rank {r}/{w}: " + "; ".join(errs)
                                + f" (transport {C.transport_summary()})")
    return {"ok": True, "world": w, "ms": round((time.perf_counter() - t0) * 1000.0, 2)}


def capture_probe(comm, agree: Agreement, rank: int) -> tuple[bool, str]:
    """Capture fork -> all_reduce -> join in a tiny hipGraph, agree, replay twice, verify, agree.
    Returns (graph_ok_on_all_ranks, reason). On a CPU communicator only the agreement (and the
    fault injection) runs: there is nothing to capture."""
    dev = comm.device
    g = y = x = None
    err = ""
    try:
        capture_fault("probe", rank)
        if dev.type == "cuda":
            x = torch.full((2048,), float(comm.rank + 1), dtype=torch.float32, device=dev)
            y = torch.empty_like(x)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                y.copy_(x)
                comm.all_reduce(y)
    except Exception as e:  # noqa: BLE001 -- every failure votes no
        err = f"capture: {type(e).__name__}: {e}"[:600]
        g = None
    ok, bad = agree.decide("probe_capture", not err, err)
    if not ok:
        return False, Agreement.summary(bad)
    if g is not None:
        want = comm.world * (comm.world + 1) / 2.0
        try:
            for _ in range(2):
                y.zero_()
                g.replay()
                torch.cuda.synchronize(dev)
                if not bool((y == want).all()):
                    raise RuntimeError(f"replayed all_reduce gave {y[0].item()} (want {want})")
        except Exception as e:  # noqa: BLE001
            err = f"replay: {type(e).__name__}: {e}"[:600]
    ok, bad = agree.decide("probe_replay", not err, err)
    return ok, "ok" if ok else Agreement.summary(bad)
