"""dropout_add_layer_norm off the GPU: the composition it stands for
(dropout_add, then the LayerNorm / its dual forms) in every mode."""
import pytest
import torch
from torch import nn

from distributed_compute_pytorch_amd.ops.dropout import dropout_add
from distributed_compute_pytorch_amd.ops.layernorm import FusedLayerNorm, dropout_add_layer_norm


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("fused_ln", [True, False])
@pytest.mark.parametrize("p,training", [(0.0, True), (0.3, False), (0.3, True)])
def test_matches_composition(mode, fused_ln, p, training):
    torch.manual_seed(0)
    ln = FusedLayerNorm(16) if fused_ln else nn.LayerNorm(16)
    br = torch.randn(3, 5, 16, requires_grad=True)
    res = torch.randn(3, 5, 16, requires_grad=True)
    torch.manual_seed(4)
    got = dropout_add_layer_norm(br, res, ln, p, training, mode)
    torch.manual_seed(4)
    x = dropout_add(br, res, p, training)
    y = ln(x)
    want = y if mode == 0 else ((y, x) if mode == 1 else (y, y))
    if mode == 0:
        torch.testing.assert_close(got, want)
    else:
        for a, b in zip(got, want):
            torch.testing.assert_close(a, b)


def test_gradients_flow_to_both_inputs():
    torch.manual_seed(1)
    ln = FusedLayerNorm(8)
    br = torch.randn(4, 8, requires_grad=True)
    res = torch.randn(4, 8, requires_grad=True)
    y, x = dropout_add_layer_norm(br, res, ln, 0.0, True, 1)
    (y.sum() + 2 * x.sum()).backward()
    # p = 0: x = res + br, so both inputs see the same gradient
    torch.testing.assert_close(br.grad, res.grad)
    assert ln.weight.grad is not None and ln.bias.grad is not None
