"""distributed_compute_pytorch_amd — an MI355X-native data-parallel training framework.

Same user-facing API as the torch.distributed / DDP training loop of
saandeepa93/distributed_compute_pytorch, rebuilt for gfx950:
native C++ store / RCCL communicator / Reducer, hand-written HIP kernels.

    import distributed_compute_pytorch_amd as dcp
    dcp.distributed.init_process_group("rccl")
    model = dcp.parallel.DistributedDataParallel(model, device_ids=[rank])
    opt = dcp.optim.Adadelta(model.parameters(), lr=1e-3)
"""
from ._ext import C as _C  # noqa: F401  (builds/loads the native extension)
from . import distributed, parallel, optim, ops, models, utils  # noqa: F401
from .parallel import DistributedDataParallel  # noqa: F401
from .utils.data import DistributedSampler  # noqa: F401

__version__ = "0.1.0"
