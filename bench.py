#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole job) of ResNet-50 bf16 MultiWorkerMirroredStrategy
training on N MI355X GPUs of one node (BASELINE.json metric/config).

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

One process per GPU (RANK/LOCAL_RANK/WORLD_SIZE from the launcher), RCCL over xGMI for the
bucketed gradient all-reduce, hand-written gfx950 HIP kernels for conv/BN/pool/loss/SGD.
Synthetic ImageNet-shaped data (on-device, fixed batch) and random-init weights. The timed
region is exactly K full training steps (forward, backward, all-reduce, fused SGD update),
bracketed by barrier + device synchronize; rank 0 prints one JSON line with the MAX over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="per-GPU batch (default: 256 ResNet, 64 BERT, 32 Transformer)")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--graph", type=int, default=-1, help="capture step in a hipGraph (default: on for 1 GPU)")
    ap.add_argument("--fp8", type=int, default=0, help="transformer models: MX-fp8 forward GEMMs")
    args = ap.parse_args()
    if not args.batch:
        args.batch = 256 if args.model.startswith("resnet") else (64 if args.model.startswith("bert") else 32)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world == 1:
        sys.exit("for --gpus > 1 launch with: python -m torch.distributed.run --nproc-per-node N "
                 "--master-addr 127.0.0.1 bench.py --gpus N")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from tensorflow_k8s_amd.models import build_model, synthetic_batch
    from tensorflow_k8s_amd.parallel.mwms import MultiWorkerMirroredStrategy
    from tensorflow_k8s_amd.runtime.optimizer import LAMB, SGD, AdamW
    from tensorflow_k8s_amd.runtime.trainer import StepRunner

    is_cnn = args.model.startswith("resnet")
    model = build_model(args.model, **({"fp8": True} if args.fp8 else {})).to(dev)
    if is_cnn:
        opt = SGD(model.arena, lr=0.1 * args.batch * world / 256, momentum=0.9, weight_decay=5e-5)
        opt_name = "SGD momentum 0.9 (fused HIP)"
    elif args.model.startswith("bert"):
        opt = LAMB(model.arena, lr=1e-4, weight_decay=0.01)
        opt_name = "LAMB (fused HIP)"
    else:
        opt = AdamW(model.arena, lr=1e-4, b2=0.98, eps=1e-9, weight_decay=0.0)
        opt_name = "Adam (fused HIP)"
    strat = MultiWorkerMirroredStrategy(model.arena, bucket_mb=args.bucket_mb)
    strat.configure_optimizer(opt)
    strat.broadcast_parameters()
    batch = synthetic_batch(model, args.batch, dev, seed=1000 + rank)
    # dropout seeds advance per step on the host -> transformer steps stay eager
    use_graph = (world == 1 and is_cnn) if args.graph < 0 else bool(args.graph)
    runner = StepRunner(model, opt, strat, batch, use_graph=use_graph)

    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1000.0
    gb = args.batch * world
    value = gb / (ms / 1000.0)
    loss = runner.last_loss()
    if rank == 0 and not is_cnn:
        seq = model.cfg.seq_len if args.model.startswith("bert") else model.cfg.tgt_len
        toks = gb * (seq if args.model.startswith("bert") else model.cfg.src_len + model.cfg.tgt_len)
        print(json.dumps({
            "metric": f"{args.model} training throughput (whole node)", "value": round(toks / (ms / 1000.0), 1),
            "unit": "tokens/sec", "sequences_per_sec": round(value, 2), "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16+mxfp8-fwd" if args.fp8 else "bf16",
            "data": "synthetic token ids, random-init weights",
            "config": {"model": args.model, "global_batch": gb, "seq_len": seq, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "strategy": "MultiWorkerMirroredStrategy (RCCL all-reduce)",
                       "optimizer": opt_name, "hipgraph": use_graph},
            "loss": loss}), flush=True)
    elif rank == 0:
        is_r50 = args.model == "resnet50"
        base = _baseline(world) if is_r50 else None
        print(json.dumps({
            "metric": ("images/sec (whole node) ResNet-50 TFJob at 1/2/4/8 MI355X workers" if is_r50
                       else f"{args.model} images/sec (whole node)"),
            "value": round(value, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / base, 4) if base else None, "dtype": "bf16",
            "data": "synthetic (on-device ImageNet-shaped 224x224x3 bf16 batch, random-init weights)",
            "config": {"model": args.model, "global_batch": gb, "seq_len": None, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "strategy": "MultiWorkerMirroredStrategy (RCCL all-reduce)",
                       "optimizer": opt_name, "hipgraph": use_graph},
            "loss": loss,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _baseline(world: int):
    """Stock PyTorch-ROCm comparator (eager, MIOpen/hipBLASLt, channels_last bf16 autocast) measured
    on MI355X by tools/stock_resnet.py and recorded in profiles/comparators.json;
    scaled by world for weak scaling. None until measured."""
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "comparators.json")) as f:
            v = json.load(f).get("resnet50_bf16_stock_pytorch_1gpu_img_s")
        return v * world if v else None
    except Exception:
        return None


if __name__ == "__main__":
    main()
