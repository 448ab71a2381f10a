"""Small-table embedding backward (embedding.hip, tables of <= 8 rows such as
BERT's token types) vs torch.nn.Embedding's gradient in fp32."""
import pytest
import torch
from torch import nn

from distributed_compute_pytorch_amd.ops.embedding import FusedEmbedding

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("V,D", [(1, 768), (2, 768), (3, 20), (8, 64), (2, 4)])
@pytest.mark.parametrize("kind", ["zeros", "rand"])
def test_small_table_grad_matches_torch(cuda, V, D, kind):
    torch.manual_seed(0)
    ref = nn.Embedding(V, D).to(cuda)
    ours = FusedEmbedding(V, D).to(cuda)
    ours.load_state_dict(ref.state_dict())
    B, T = 7, 301
    idx = torch.zeros(B, T, dtype=torch.long, device=cuda) if kind == "zeros" else torch.randint(0, V, (B, T), device=cuda)
    for _ in range(2):  # the second backward accumulates into the existing .grad
        g = torch.randn(B, T, D, device=cuda)
        ref(idx).backward(g)
        ours(idx).backward(g)
    torch.testing.assert_close(ours.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)


def test_small_table_kernel_direct(cuda):
    from distributed_compute_pytorch_amd._ext import C

    g = torch.randn(16384, 768, device=cuda)
    idx = torch.randint(0, 2, (16384,), device=cuda)
    gw = torch.ones(2, 768, device=cuda)
    C.embedding_small_bwd(idx, g, gw)
    want = torch.ones(2, 768, device=cuda)
    want.index_add_(0, idx, g)
    torch.testing.assert_close(gw, want, rtol=1e-4, atol=1e-3)
