"""Checkpoint / resume.

The reference saves only ``model.state_dict()`` from every rank to
``mnist.pt`` (main.py:133), racing on the file. Here:

* :func:`save_model` — rank 0 only, after a barrier, atomic rename; the layout
  is the plain torch state_dict (``module.`` prefix when DDP-wrapped), loadable
  by stock ``torch.load(weights_only=True)``.
* :func:`save_checkpoint` / :func:`load_checkpoint` — full training state:
  model, optimizer (torch-compatible ``state``/``param_groups``), scheduler,
  epoch/step, sampler epoch and RNG states; resume restores all of it.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch

from .. import distributed as dist


def _atomic_save(obj, path: str):
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_model(model: torch.nn.Module, path: str) -> None:
    if dist.is_initialized():
        dist.barrier()
    if dist.get_rank() == 0:
        _atomic_save(model.state_dict(), path)
    if dist.is_initialized():
        dist.barrier()


def save_checkpoint(path: str, model, optimizer=None, scheduler=None, epoch: int = 0, step: int = 0,
                    extra: Optional[Dict[str, Any]] = None) -> None:
    if dist.is_initialized():
        dist.barrier()
    if dist.get_rank() == 0:
        state = {
            "model": model.state_dict(),
            "optimizer": optimizer.state_dict() if optimizer is not None else None,
            "scheduler": scheduler.state_dict() if scheduler is not None else None,
            "epoch": epoch,
            "step": step,
            "rng_cpu": torch.get_rng_state(),
            "rng_cuda": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else None,
            "extra": extra or {},
        }
        _atomic_save(state, path)
    if dist.is_initialized():
        dist.barrier()


def load_checkpoint(path: str, model, optimizer=None, scheduler=None, map_location=None) -> Dict[str, Any]:
    # weights_only=True: checkpoints are plain tensors / containers (no code)
    state = torch.load(path, map_location=map_location or "cpu", weights_only=True)
    model.load_state_dict(state["model"])
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if scheduler is not None and state.get("scheduler") is not None:
        scheduler.load_state_dict(state["scheduler"])
    if state.get("rng_cpu") is not None:
        torch.set_rng_state(state["rng_cpu"])
    if state.get("rng_cuda") is not None and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(state["rng_cuda"])
    return {"epoch": state.get("epoch", 0), "step": state.get("step", 0), "extra": state.get("extra", {})}
