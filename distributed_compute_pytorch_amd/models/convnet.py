"""The reference model: MNIST ConvNet (main.py:20-45).

conv(1→32,k3) → ReLU → conv(32→64,k3) → ReLU → maxpool2 → Dropout2d(0.25)
→ flatten(9216) → fc(9216→128) → BatchNorm1d(128) → ReLU → dropout(0.5)
→ fc(128→10) → log_softmax.  1,200,138 parameters, 3 BN buffers.

Parameter registration order and names match the reference exactly
(conv1, conv2, dropout1, dropout2, fc1, fc2, batchnorm), so state_dict keys —
``module.conv1.weight`` … ``module.batchnorm.num_batches_tracked`` under DDP —
are identical. The reference applies ``Dropout2d`` to the 2-D
fc1 activation, which acts element-wise; ``nn.Dropout`` is
used for ``dropout2`` so behaviour is the same without the 2.x warning.

``fused=True`` (GPU) runs the MI355X path with identical parameters and
state_dict: conv1 → ReLU → conv2 → ReLU → max-pool → Dropout2d → flatten as
ONE fp32-MFMA kernel forward and one (+ reduce) backward
(``ops/convnet.py``, ``csrc/kernels/convnet.hip``), fc1 / fc2 on fp32-MFMA
GEMMs (``csrc/kernels/fc32.hip``: K-split forward, data gradient, weight
gradient with the bias gradient in the same launch), [BatchNorm1d + ReLU] on
the fused BN kernels, Philox dropout, and a wave-per-row log-softmax
(SURVEY §2f K1-K6, K8-K13, K16-K24).
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F

from ..ops.batchnorm import BatchNormAct1d


class ConvNet(nn.Module):
    def __init__(self, fused: bool = False):
        super().__init__()
        self.fused = fused
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout2d(0.25)
        self.dropout2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)
        self.batchnorm = BatchNormAct1d(128, act=fused, fused=fused)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.fused and x.is_cuda:
            return self._forward_fused(x)
        x = F.relu(self.conv1(x))
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = self.fc1(x)
        x = self.batchnorm(x)
        x = F.relu(x)
        x = self.dropout2(x)
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)

    def _forward_fused(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops import convnet_features, fc32, fused_dropout, fused_log_softmax

        x = convnet_features(x, self.conv1, self.conv2, self.dropout1.p, self.training)
        x = self.batchnorm(fc32(x, self.fc1))  # fp32-MFMA fc1, then BN1d + ReLU
        x = fused_dropout(x, self.dropout2.p, self.training)
        return fused_log_softmax(fc32(x, self.fc2), 1)
