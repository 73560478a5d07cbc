"""Step runner: eager or hipGraph-captured training step (forward + backward + gradient
all-reduce + fused optimizer).

hipGraph (``torch.cuda.CUDAGraph`` on ROCm) removes the ~600 host launches of a ResNet-50 step:
after two eager warm-up steps (which also size every workspace) the whole step is captured once
and replayed -- at every world size: the data-parallel strategies enqueue their RCCL collectives
(parallel/tfk_comm.py) on a comm stream forked from the capturing stream at the moment backward
produces each bucket, so the replayed graph keeps the bucket/backward overlap.

Everything a replay must see change per step lives on the device: the optimizer's learning-rate
schedule, step counter and Adam bias corrections (Optimizer.enable_device_schedule) and the models'
dropout RNG state (ops.elementwise.rng_advance/rng_key). Host-side per-step values that would
freeze inside a graph make capture refuse (GraphUnsafe) instead of silently training wrong.

Multi-rank safety (runtime/guard.py): with an ``agree`` (guard.Agreement over the ranks that share
the step's collectives) the capture result is voted on before the first replay; if any rank failed
to capture, every rank drops its graph and the step runs eagerly from then on (``fallback`` holds
the reason) -- nobody is left waiting in a replayed collective its peer never issues.
"""
from __future__ import annotations

import torch


class GraphUnsafe(RuntimeError):
    """The step has host-side per-step state a captured graph would freeze."""


def graph_hazards(model) -> list[str]:
    """Reasons a model's step cannot be replayed from a hipGraph (empty = safe). Dropout is safe when
    the model keeps its RNG state on the device (``rng_state``, advanced inside the step)."""
    out = []
    cfg = getattr(model, "cfg", None)
    if getattr(model, "rng_state", None) is not None:
        return out
    for k in ("dropout", "hidden_dropout", "attn_dropout", "relu_dropout"):
        if cfg is not None and float(getattr(cfg, k, 0.0) or 0.0) > 0.0 and getattr(model, "training", True):
            out.append(f"{type(model).__name__}.cfg.{k}={getattr(cfg, k)} (dropout seeds are drawn on the host per step)")
    return out


class StepRunner:
    def __init__(self, model, opt, strategy, batch, use_graph: bool = False, warmup_eager: int = 2,
                 agree=None, rank: int = 0):
        self.model, self.opt, self.strategy = model, opt, strategy
        self.batch = batch
        # a parameter-server strategy is capturable only on its collective (RCCL) transport
        self.use_graph = (use_graph and torch.cuda.is_available() and batch[0].is_cuda
                          and (not hasattr(strategy, "apply_gradients") or getattr(strategy, "capturable", False)))
        self.fallback = ""  # why the step runs eager (refused or failed capture)
        if self.use_graph:
            bad = graph_hazards(model)
            if bad:
                raise GraphUnsafe("hipGraph capture refused: " + "; ".join(bad))
            if opt is not None and hasattr(opt, "enable_device_schedule"):
                opt.enable_device_schedule()
        self.warmup_eager = warmup_eager
        self.agree, self.rank = agree, rank
        self.graph = None
        self.n = 0
        self._loss = None
        self._corr = None

    def _step_body(self):
        s = self.strategy
        if s is not None:
            s.begin_step()
        loss, corr = self.model.forward_backward(*self.batch)
        if s is not None:
            s.finish_step()
        if s is not None and hasattr(s, "apply_gradients"):
            s.apply_gradients(self.opt)  # parameter-server: the update runs on the ps tasks
        else:
            self.opt.step()
        return loss, corr

    def set_batch(self, *tensors):
        """Copy a new batch into the static input buffers (keeps captured graphs valid)."""
        for dst, src in zip(self.batch, tensors):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)

    def step(self):
        self.n += 1
        if not self.use_graph:
            self._loss, self._corr = self._step_body()
            return
        if self.graph is None:
            if self.n <= self.warmup_eager:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    self._loss, self._corr = self._step_body()
                torch.cuda.current_stream().wait_stream(side)
                return
            if not self._capture():
                self._loss, self._corr = self._step_body()  # agreed fallback: this step runs eager
                return
        self.graph.replay()

    def _capture(self) -> bool:
        from .guard import Agreement, capture_fault
        err = ""
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        try:
            capture_fault("step", self.rank)
            # thread-local capture: a watchdog thread polling RCCL / events while this thread
            # captures must not invalidate the capture (the default global mode would)
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._loss, self._corr = self._step_body()
        except Exception as e:  # noqa: BLE001 -- every failure votes no
            err = f"{type(e).__name__}: {e}"[:600]
            if self.agree is None:
                raise
        ok = not err
        if self.agree is not None:
            ok, bad = self.agree.decide("step_capture", not err, err)
            if not ok:
                err = Agreement.summary(bad)
        if not ok:
            self.graph, self.use_graph, self.fallback = None, False, err
            del g
            torch.cuda.synchronize()
            from . import streams
            streams.reset()  # weight gradients queued by the aborted capture must never run
            return False
        self.graph = g
        return True

    def last_loss(self):
        if self._loss is None:
            return None
        return float(self._loss.float().mean().item())

    def last_accuracy(self):
        if self._corr is None:
            return None
        return float(self._corr.float().mean().item())
