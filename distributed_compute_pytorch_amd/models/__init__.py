"""Model zoo: the reference ConvNet, an MLP, ResNet-50 (+BERT-base, GPT-2-small)."""
from .convnet import ConvNet
from .mlp import MLP
from .resnet import ResNet, resnet50, resnet18_like

__all__ = ["ConvNet", "MLP", "ResNet", "resnet50", "resnet18_like"]
