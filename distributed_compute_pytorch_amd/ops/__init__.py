"""Hand-written gfx950 ops exposed as torch modules / autograd functions."""
from .batchnorm import BatchNormAct2d, bn_act

__all__ = ["BatchNormAct2d", "bn_act"]
