"""Evaluator replica (TFJob replica type "Evaluator").

Not part of the training world: follows the chief's checkpoint directory, and for every new
checkpoint restores it into an inference copy of the model (BN in moving-statistics mode) and
reports loss/accuracy on a fixed synthetic evaluation set. Exits when the final checkpoint
(marked by ``<dir>/DONE``) has been evaluated, or after ``--eval-timeout`` seconds without one.
"""
from __future__ import annotations

import json
import os
import time

import torch


def evaluate(model, batches) -> dict:
    from ..ops.loss import softmax_xent
    tot_loss, tot_corr, n = 0.0, 0.0, 0
    if hasattr(model, "evaluate"):  # sequence models: (loss sum, hits, predictions) per batch
        for b in batches:
            l_, c_, n_ = model.evaluate(*b)
            tot_loss, tot_corr, n = tot_loss + l_, tot_corr + c_, n + n_
        return {"loss": tot_loss / max(n, 1), "accuracy": tot_corr / max(n, 1), "examples": n}
    model.train(False)
    for x, y in batches:
        logits = model.forward(x)
        loss, _, corr = softmax_xent(logits, y, want_grad=False, want_correct=True)
        tot_loss += float(loss.sum())
        tot_corr += float(corr.sum())
        n += int(y.numel())
    model.train(True)
    return {"loss": tot_loss / max(n, 1), "accuracy": tot_corr / max(n, 1), "examples": n}


def run_evaluator(args) -> int:
    from ..models import build_model, synthetic_batch
    from .checkpoint import CheckpointManager
    from .train import data_kwargs, model_kwargs
    if not args.checkpoint_dir:
        print(json.dumps({"event": "error", "message": "evaluator needs --checkpoint-dir"}), flush=True)
        return 1
    dev = torch.device("cuda", 0) if (args.device != "cpu" and torch.cuda.is_available()) else torch.device("cpu")
    model = build_model(args.model, **model_kwargs(args)).to(dev, seed=args.seed)
    batches = [synthetic_batch(model, args.batch, dev, seed=10_000_019 + i, **data_kwargs(args))
               for i in range(max(1, args.eval_batches))]
    mgr = CheckpointManager(args.checkpoint_dir, args.keep)
    seen = set()
    deadline = time.time() + args.eval_timeout
    from . import health
    while True:
        health.beat()
        latest = mgr.latest()
        if latest is not None and latest not in seen:
            seen.add(latest)
            step = mgr.restore(model.arena, None, latest, strict=True)
            res = evaluate(model, batches)
            print(json.dumps({"event": "eval", "step": step, "checkpoint": os.path.basename(latest), **res},
                             sort_keys=True), flush=True)
            deadline = time.time() + args.eval_timeout
        done = os.path.join(args.checkpoint_dir, "DONE")
        if os.path.exists(done):
            final = open(done).read().strip()
            if latest is not None and latest.endswith(f"-{final}"):
                print(json.dumps({"event": "done", "role": "evaluator", "evaluated": len(seen)}), flush=True)
                return 0
        if time.time() > deadline:
            print(json.dumps({"event": "error", "message": "evaluator timed out waiting for checkpoints"}), flush=True)
            return 1
        time.sleep(0.5)
