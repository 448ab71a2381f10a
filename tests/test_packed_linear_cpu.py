"""ops.linear.packed_linear (BERT's packed query/key/value projection): same
output and per-layer parameter gradients as the separate Linears (CPU path:
one F.linear over the autograd-concatenated weights)."""
import torch
from torch import nn

from distributed_compute_pytorch_amd.ops.linear import packed_linear


def test_packed_linear_matches_separate_layers():
    torch.manual_seed(0)
    layers = [nn.Linear(32, 32) for _ in range(3)]
    ref = [nn.Linear(32, 32) for _ in range(3)]
    for a, b in zip(layers, ref):
        b.load_state_dict(a.state_dict())
    x = torch.randn(4, 7, 32, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    y = packed_linear(x, layers)
    yr = torch.cat([l(xr) for l in ref], -1)
    torch.testing.assert_close(y, yr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad)
    for a, b in zip(layers, ref):
        torch.testing.assert_close(a.weight.grad, b.weight.grad)
        torch.testing.assert_close(a.bias.grad, b.bias.grad)


def test_bert_state_dict_keys_unchanged():
    from distributed_compute_pytorch_amd.models.bert import BertConfig, BertForPreTraining

    m = BertForPreTraining(BertConfig(vocab_size=64, hidden=64, layers=1, heads=2, intermediate=128, max_position=16,
                                      fused=True))
    keys = set(m.state_dict())
    assert {"layers.0.attention.query.weight", "layers.0.attention.key.weight",
            "layers.0.attention.value.bias"} <= keys, sorted(keys)[:20]
