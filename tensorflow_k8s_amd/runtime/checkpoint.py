"""TF-layout checkpoints for the tfk executor.

Writes TensorFlow V2 tensor bundles through the native C++ writer (cpp/runtime/tfbundle.cc via
tensorflow_k8s_amd._C): `<dir>/model.ckpt-<step>.index`, `.data-00000-of-00001` and the text
`checkpoint` state file, chief only, with TF variable names and layouts (conv kernels HWIO,
dense [in, out], BN gamma/beta/moving_mean/moving_variance, optimizer slots `<var>/Momentum`,
`<var>/Adam`, `<var>/Adam_1`, and `global_step`). Checkpoints are world-size independent, so a
job resumes after restarts or a scale change. Saves are asynchronous: one device->host snapshot
on the calling stream, then the file write on a background thread; the write is atomic
(tmp + fsync + rename) and `checkpoint` is rewritten last. Keeps the newest `max_to_keep`.
"""
from __future__ import annotations

import glob
import os
import threading

import numpy as np
import torch

from ..ops._lib import lib

SLOT_SUFFIX = {"Momentum": "Momentum", "Adam": "Adam", "Adam_1": "Adam_1"}
# fault injection (tests): seconds every asynchronous checkpoint write stalls before writing
FAULT_WRITE_DELAY_S = float(os.environ.get("TFK_FAULT_CKPT_DELAY_S", "0"))


class CheckpointWriteError(RuntimeError):
    """A checkpoint could not be written (e.g. the disk is full). The previous checkpoint and the
    `checkpoint` state file are untouched (tmp + rename), so a restart resumes from it."""


def _to_tf(p, arr: np.ndarray) -> np.ndarray:
    return p.spec.to_tf(arr) if p.spec.to_tf is not None else arr


def _from_tf(p, arr: np.ndarray) -> np.ndarray:
    return p.spec.from_tf(arr) if p.spec.from_tf is not None else arr


class CheckpointManager:
    def __init__(self, directory: str, max_to_keep: int = 5, prefix: str = "model.ckpt"):
        self.dir = directory
        self.max_to_keep = max_to_keep
        self.prefix = prefix
        self._thread: threading.Thread | None = None
        self.error: Exception | None = None
        os.makedirs(directory, exist_ok=True)

    # ------------------------------------------------------------------ save
    def snapshot(self, arena, optimizer=None, step: int = 0, extra: dict | None = None) -> dict:
        """Device -> host copies of everything to save, keyed by TF variable name."""
        host_master = arena.master.detach().to("cpu", non_blocking=False)
        out = {}
        for p in arena.params:
            a = host_master[p.offset:p.offset + p.numel].numpy().reshape(p.spec.shape)
            out[p.name] = np.ascontiguousarray(_to_tf(p, a))
        if optimizer is not None:
            for slot in optimizer.slot_names:
                hs = arena.slot(slot).detach().cpu()
                for p in arena.params:
                    a = hs[p.offset:p.offset + p.numel].numpy().reshape(p.spec.shape)
                    out[f"{p.name}/{SLOT_SUFFIX.get(slot, slot)}"] = np.ascontiguousarray(_to_tf(p, a))
        for b in arena.buffers:
            t = b.tensor.detach().cpu().numpy()
            out[b.name] = np.ascontiguousarray(b.to_tf(t) if b.to_tf else t)
        out["global_step"] = np.asarray(step, dtype=np.int64)
        for k, v in (extra or {}).items():
            out[k] = np.asarray(v)
        return out

    def save(self, arena, optimizer=None, step: int = 0, extra: dict | None = None, blocking: bool = False) -> str:
        self.wait()
        tensors = self.snapshot(arena, optimizer, step, extra)
        name = f"{self.prefix}-{step}"

        def work():
            try:
                if FAULT_WRITE_DELAY_S > 0:
                    import time
                    time.sleep(FAULT_WRITE_DELAY_S)  # fault injection: a slow disk
                names = sorted(tensors)
                lib().ckpt_write(os.path.join(self.dir, name), names, [torch.from_numpy(tensors[n]) for n in names])
                existing = self.all_checkpoints()
                if name not in existing:
                    existing.append(name)
                keep = existing[-self.max_to_keep:]
                lib().ckpt_state_write(self.dir, name, keep)
                for old in existing[:-self.max_to_keep]:
                    for f in glob.glob(os.path.join(self.dir, old + ".*")):
                        os.remove(f)
            except Exception as e:  # surfaced by wait()
                self.error = CheckpointWriteError(f"checkpoint {name} not written: {e}")

        if blocking:
            work()
            self._raise()
        else:
            self._thread = threading.Thread(target=work, daemon=True)
            self._thread.start()
        return os.path.join(self.dir, name)

    def wait(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        self._raise()

    def _raise(self):
        if self.error is not None:
            e, self.error = self.error, None
            raise e

    # ------------------------------------------------------------------ restore
    def latest(self) -> str | None:
        latest, _ = lib().ckpt_state_read(self.dir) if os.path.exists(os.path.join(self.dir, "checkpoint")) else ("", [])
        if not latest:
            return None
        p = latest if os.path.isabs(latest) else os.path.join(self.dir, latest)
        return p if os.path.exists(p + ".index") else None

    def all_checkpoints(self) -> list:
        if not os.path.exists(os.path.join(self.dir, "checkpoint")):
            return []
        _, all_ = lib().ckpt_state_read(self.dir)
        return [a for a in all_ if os.path.exists(os.path.join(self.dir, a + ".index"))]

    def restore(self, arena, optimizer=None, path: str | None = None, strict: bool = True) -> int | None:
        """Loads a checkpoint into the arena (master -> compute refreshed). Returns global_step."""
        path = path or self.latest()
        if path is None:
            return None
        tensors = lib().ckpt_read(path)
        host = arena.master.detach().cpu().clone()
        missing = []
        for p in arena.params:
            t = tensors.get(p.name)
            if t is None:
                missing.append(p.name)
                continue
            a = _from_tf(p, t.float().numpy())
            host[p.offset:p.offset + p.numel] = torch.from_numpy(np.ascontiguousarray(a)).reshape(-1)
        if missing and strict:
            raise KeyError(f"checkpoint {path} lacks {len(missing)} variables, e.g. {missing[:3]}")
        arena.master.copy_(host)
        arena.refresh_compute()
        if optimizer is not None:
            for slot in optimizer.slot_names:
                hs = arena.slot(slot).detach().cpu().clone()
                for p in arena.params:
                    t = tensors.get(f"{p.name}/{SLOT_SUFFIX.get(slot, slot)}")
                    if t is not None:
                        hs[p.offset:p.offset + p.numel] = torch.from_numpy(
                            np.ascontiguousarray(_from_tf(p, t.float().numpy()))).reshape(-1)
                arena.slot(slot).copy_(hs)
        for b in arena.buffers:
            t = tensors.get(b.name)
            if t is not None:
                b.tensor.copy_(t.to(b.tensor.dtype).reshape(b.tensor.shape))
        step = int(tensors["global_step"]) if "global_step" in tensors else 0
        if optimizer is not None:
            optimizer.step_count = step
        return step
