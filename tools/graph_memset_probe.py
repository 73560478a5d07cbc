#!/usr/bin/env python3
"""Fault-free probe of the round-4/5 captured-step fault hypothesis: is a hipMemsetAsync captured into
a hipGraph ordered before the kernels that follow it on replay, when the graph also forks onto a
second stream (the RCCL comm stream of the data-parallel strategies)?

The graph mirrors the embedding backward's shape: memset(cnt) -> count kernel (index_add_ of ones
at valid token ids: never out of range) -> [a fork onto a side stream with an optional world-1 RCCL
all-reduce, joined later] -> more main-stream work. After every replay cnt must equal bincount(ids);
a stale or racing memset shows up as wrong counts, not as a GPU fault.

    python tools/graph_memset_probe.py [--replays 50]
prints one JSON line per variant: {"variant", "replays", "bad_replays", "max_err"}.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def hip_memset_async():
    lib = ctypes.CDLL("libamdhip64.so")
    fn = lib.hipMemsetAsync
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    return fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    memset = hip_memset_async()
    V, ntok = 33728, 8192
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, V, (ntok,), generator=g).to(dev)
    ref = torch.bincount(ids, minlength=V).to(torch.int32)
    ones = torch.ones(ntok, dtype=torch.int32, device=dev)
    cnt = torch.zeros(V, dtype=torch.int32, device=dev)
    filler = torch.randn(4096, 4096, device=dev)
    comm = None
    try:
        import torch.distributed as dist

        from tensorflow_k8s_amd.parallel import tfk_comm
        comm = tfk_comm.init(dist.HashStore(), 0, 1, dev)
    except Exception as e:  # noqa: BLE001 -- the RCCL variant is skipped
        print(json.dumps({"note": f"no world-1 RCCL communicator: {e}"[:300]}), flush=True)
    buf = torch.zeros(1 << 20, device=dev)

    def body(variant):
        s = torch.cuda.current_stream()
        if variant != "plain":
            side = comm.stream if (variant == "rccl" and comm is not None) else SIDE
            side.wait_stream(s)
            if variant == "rccl" and comm is not None:
                comm._c.all_reduce(buf, buf, "sum", side.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(side)
        rc = memset(ctypes.c_void_p(cnt.data_ptr()), 0, cnt.numel() * 4, ctypes.c_void_p(s.cuda_stream))
        assert rc == 0, rc
        cnt.index_add_(0, ids, ones)
        filler.mul_(1.0000001)  # more main-stream work after the counts
        if variant != "plain":
            s.wait_event(ev)

    SIDE = torch.cuda.Stream(device=dev)
    variants = ["plain", "fork"] + (["rccl"] if comm is not None else [])
    for v in variants:
        for _ in range(2):  # eager warm-up
            body(v)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            body(v)
        bad, worst = 0, 0
        for _ in range(args.replays):
            cnt.fill_(7)  # poison outside the graph: only a working memset node restores the counts
            gr.replay()
            torch.cuda.synchronize()
            err = int((cnt - ref).abs().max())
            bad += err != 0
            worst = max(worst, err)
        print(json.dumps({"variant": v, "replays": args.replays, "bad_replays": bad, "max_err": worst}), flush=True)
        del gr
    if comm is not None:
        tfk_comm.shutdown()


if __name__ == "__main__":
    main()
