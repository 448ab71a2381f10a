"""Fused optimizers (torch-compatible state) + LR schedulers.

LR schedulers are optimizer-agnostic in torch, so torch's ``StepLR`` (the
reference's scheduler, main.py:125) drives these optimizers unchanged.
"""
from torch.optim.lr_scheduler import StepLR, CosineAnnealingLR, LambdaLR, LinearLR, OneCycleLR  # noqa: F401

from .fused import SGD, Adam, AdamW, Adadelta, clip_grad_norm_

__all__ = ["SGD", "Adam", "AdamW", "Adadelta", "clip_grad_norm_", "StepLR", "CosineAnnealingLR", "LambdaLR",
           "LinearLR", "OneCycleLR"]
