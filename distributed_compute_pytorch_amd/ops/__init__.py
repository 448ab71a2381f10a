"""Hand-written gfx950 ops exposed as torch modules / autograd functions."""
from .batchnorm import BatchNormAct1d, BatchNormAct2d, bn_act
from .layernorm import FusedLayerNorm, fused_layer_norm
from .cross_entropy import fused_cross_entropy
from .metrics import EvalMetrics
from .pool import FusedMaxPool2d, fused_max_pool2d, relu_max_pool2d_dropout
from .dropout import FusedDropout, FusedDropout2d, dropout_add, fused_dropout, fused_feature_dropout
from .softmax import fused_log_softmax
from .convnet import convnet_features, fc32

__all__ = ["BatchNormAct1d", "BatchNormAct2d", "bn_act", "FusedLayerNorm", "fused_layer_norm", "fused_cross_entropy",
           "FusedDropout", "FusedDropout2d", "dropout_add", "fused_dropout", "fused_feature_dropout",
           "FusedMaxPool2d", "fused_max_pool2d", "relu_max_pool2d_dropout", "fused_log_softmax", "EvalMetrics",
           "convnet_features", "fc32"]
