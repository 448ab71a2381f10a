"""Utilities: data (sampler, synthetic batches), metrics/timers, checkpointing."""
from .data import DistributedSampler, SyntheticBatches, SyntheticDataset, MNISTIdx
from .metrics import StepTimer, JsonLogger, print0
from .checkpoint import save_model, save_checkpoint, load_checkpoint

__all__ = ["DistributedSampler", "SyntheticBatches", "SyntheticDataset", "MNISTIdx", "StepTimer", "JsonLogger",
           "print0", "save_model", "save_checkpoint", "load_checkpoint"]
