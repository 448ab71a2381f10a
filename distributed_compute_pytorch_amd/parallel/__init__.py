"""Data-parallel engine: DistributedDataParallel + comm hooks + helpers."""
from .ddp import (DistributedDataParallel, GradBucket, DEFAULT_BUCKET_CAP_MB, DEFAULT_FIRST_BUCKET_MB,
                  XGMI_BUCKETS)
from . import comm_hooks
from .comm_utils import broadcast_coalesced, verify_params_across_processes

DDP = DistributedDataParallel

__all__ = ["DistributedDataParallel", "DDP", "GradBucket", "comm_hooks", "broadcast_coalesced",
           "verify_params_across_processes", "DEFAULT_BUCKET_CAP_MB", "DEFAULT_FIRST_BUCKET_MB",
           "XGMI_BUCKETS"]
