"""8-wave ping-pong 256 x 256 GEMM (csrc/kernels/gemm_pp.hip) vs an fp32
PyTorch reference of the same op on the same bf16 operands: plain, + bias,
+ bias + GELU (tanh / erf, computed from the bf16-rounded pre-activation),
with M / N tails (rows and columns past the tile clamp on load and are not
stored), K from one to many 64-deep K-tiles (the DMA schedule's tail runs
into the sink), and a strided output (ldc > N)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, w, b):
    y = x.float() @ w.float().t()
    return y + b if b is not None else y


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


SHAPES = [(256, 256, 64), (512, 768, 768), (1000, 264, 128), (37, 520, 192), (4096, 3072, 768),
          (777, 2304, 3072), (256, 4096, 640), (16384, 768, 3072)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("mode", ["plain", "bias", "gelu_tanh", "gelu_erf"])
def test_gemm_pp_matches_fp32(cuda, M, N, K, mode):
    from distributed_compute_pytorch_amd._ext import C

    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    x = (torch.rand(M, K, generator=g) * 2 - 1).to(cuda).to(torch.bfloat16)
    w = ((torch.rand(N, K, generator=g) * 2 - 1) / K ** 0.5).to(cuda).to(torch.bfloat16)
    b = (torch.rand(N, generator=g) - 0.5).to(cuda) if mode != "plain" else None
    gelu = {"plain": 0, "bias": 0, "gelu_tanh": 1, "gelu_erf": 2}[mode]
    out = C.gemm_pp(x, w, b, gelu)
    ref = _ref(x, w, b)
    if gelu:
        act, h = out
        assert h.dtype == torch.bfloat16 and act.shape == (M, N)
        assert _rel(h, ref) < 5e-3, _rel(h, ref)
        # gelu from the bf16 h (what the backward reads), to bf16 rounding
        want = F.gelu(h.float(), approximate="tanh" if gelu == 1 else "none")
        torch.testing.assert_close(act.float(), want, rtol=1.6e-2, atol=1e-2)
    else:
        (y,) = out
        assert y.dtype == torch.bfloat16 and y.shape == (M, N)
        assert _rel(y, ref) < 5e-3, _rel(y, ref)
        # every element, not just the norm: a mis-staged tile stands out here
        err = (y.float() - ref).abs()
        assert float(err.max()) <= 2e-2 * float(ref.abs().max()) + 1e-2


def test_gemm_pp_repeatable_and_asymmetric(cuda):
    """Bit-identical across launches (no data race in the DMA schedule) and
    not transposed: A = I picks B's rows."""
    from distributed_compute_pytorch_amd._ext import C

    g = torch.Generator().manual_seed(5)
    x = torch.randn(2048, 1024, generator=g).to(cuda).to(torch.bfloat16)
    w = torch.randn(1536, 1024, generator=g).to(cuda).to(torch.bfloat16)
    y0 = C.gemm_pp(x, w)[0]
    for _ in range(5):
        assert torch.equal(C.gemm_pp(x, w)[0], y0)
    eye = torch.eye(256, 1024, device=cuda, dtype=torch.bfloat16)
    assert torch.equal(C.gemm_pp(eye, w)[0], w[:, :256].t().contiguous())
