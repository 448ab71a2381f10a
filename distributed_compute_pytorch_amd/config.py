"""Training configuration: one dataclass, CLI overrides.

The reference has six argparse flags (main.py:138-145: --batch_size --lr
--epochs --no-cuda --gamma --gpus). They keep their names and defaults here;
the framework-level knobs the survey lists are added next to them.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
from dataclasses import dataclass
from typing import Optional


@dataclass
class TrainConfig:
    # reference flags (main.py:139-144)
    batch_size: int = 128
    lr: float = 1e-3
    epochs: int = 20
    no_cuda: bool = False
    gamma: float = 0.7
    gpus: int = 4
    # framework knobs
    model: str = "convnet"                # convnet | mlp | resnet50 | bert | gpt2
    backend: str = "auto"                 # rccl | host | auto  (nccl / gloo aliases)
    dtype: str = "fp32"                   # fp32 | bf16 (autocast)
    steps_per_epoch: int = 0              # 0 = one pass over the sampler
    synthetic: bool = True
    data_dir: str = "./data"
    bucket_cap_mb: Optional[float] = None
    first_bucket_mb: Optional[float] = None
    gradient_as_bucket_view: bool = True
    broadcast_buffers: bool = True
    find_unused_parameters: bool = False
    comm_dtype: str = "fp32"              # fp32 | bf16 wire compression
    grad_accum: int = 1
    clip_grad_norm: float = 0.0
    hip_graph: bool = False               # capture the whole step in one HIP graph (GPU)
    seed: int = 0
    log_every: int = 10
    metrics_file: Optional[str] = None    # JSON-lines metrics (rank 0)
    checkpoint: Optional[str] = None      # full checkpoint path (save every epoch)
    resume: Optional[str] = None
    save_model: Optional[str] = "model.pt"
    profile: bool = False                 # torch.profiler chrome trace of the first epoch

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), sort_keys=True)


def _add(ap: argparse.ArgumentParser, f: dataclasses.Field):
    name = "--" + f.name.replace("_", "-")
    alias = ["--" + f.name] if "_" in f.name else []
    default = f.default if f.default is not dataclasses.MISSING else f.default_factory()
    if f.type in ("bool", bool):
        ap.add_argument(name, *alias, dest=f.name, type=lambda v: str(v).lower() in ("1", "true", "yes", "on"),
                        nargs="?", const=True, default=default)
    elif f.type in ("int", int):
        ap.add_argument(name, *alias, dest=f.name, type=int, default=default)
    elif f.type in ("float", float):
        ap.add_argument(name, *alias, dest=f.name, type=float, default=default)
    elif "Optional[float]" in str(f.type):
        ap.add_argument(name, *alias, dest=f.name, type=float, default=default)
    elif "List" in str(f.type):
        ap.add_argument(name, *alias, dest=f.name, nargs="*", default=default)
    else:
        ap.add_argument(name, *alias, dest=f.name, default=default)


def parse_config(argv=None, **defaults) -> TrainConfig:
    """CLI → TrainConfig. Accepts both --batch-size and the reference's --batch_size."""
    ap = argparse.ArgumentParser(description="distributed_compute_pytorch_amd trainer")
    for f in dataclasses.fields(TrainConfig):
        _add(ap, f)
    ap.set_defaults(**defaults)
    ns = ap.parse_args(argv)
    return TrainConfig(**vars(ns))
