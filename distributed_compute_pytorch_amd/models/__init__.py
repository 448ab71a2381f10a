"""Model zoo: the reference ConvNet, an MLP, ResNet-50, BERT-base, GPT-2-small."""
from .convnet import ConvNet
from .mlp import MLP
from .resnet import ResNet, resnet50, resnet18_like
from .gpt2 import GPT2, GPT2Config, gpt2_small
from .bert import BertForPreTraining, BertConfig, bert_base

__all__ = ["ConvNet", "MLP", "ResNet", "resnet50", "resnet18_like", "GPT2", "GPT2Config", "gpt2_small",
           "BertForPreTraining", "BertConfig", "bert_base"]
