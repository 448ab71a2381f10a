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


# persistent grid: ≤ 256 workgroups stream several tiles each once tiles > 256
# (K = 64 / 128: one / two K-tiles per tile, so the DMA runs 1-2 tiles ahead
# across tile boundaries; N % 4 tails; M tails)
SHAPES = [(256, 256, 64), (512, 768, 768), (8192, 768, 768), (300, 200, 128), (1000, 264, 128), (37, 520, 192), (4096, 3072, 768),
          (777, 2304, 3072), (256, 4096, 640), (16384, 768, 3072), (8192, 2304, 768), (9000, 2052, 128),
          (262144, 256, 64), (100352, 1024, 256), (3001, 4100, 320)]


@pytest.fixture(params=["default", "tile256", "persistent", "persistent_regepi", "pq"])
def pp_variant(request):
    """default: the automatic tile choice (gemm_pq_pick: 128 x 192 where it
    fills the chip better, else 256 x 256); tile256: always the single-tile
    256 x 256 kernel; persistent: the persistent 256 x 256 kernel for every
    grid; _regepi: every tile's epilogue from the registers; pq: always the
    128 x 192 kernel (gemm_pq.hip) where the shape is supported."""
    from distributed_compute_pytorch_amd._ext import C

    v1, stage, tile = {"default": (1, 1, 0), "tile256": (1, 1, 1), "persistent": (0, 1, 1),
                       "persistent_regepi": (0, 0, 1), "pq": (1, 1, 2)}[request.param]
    C.gemm_tune("pp_v1", v1)
    C.gemm_tune("pp_stage", stage)
    C.gemm_tune("pp_tile", tile)
    yield request.param
    C.gemm_tune("pp_v1", 1)
    C.gemm_tune("pp_stage", 1)
    C.gemm_tune("pp_tile", 0)


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("mode", ["plain", "bias", "gelu_tanh", "gelu_erf"])
def test_gemm_pp_matches_fp32(cuda, M, N, K, mode, pp_variant):
    from distributed_compute_pytorch_amd._ext import C

    gd = torch.Generator(device=cuda).manual_seed(M * 7 + N * 3 + K)
    x = (torch.rand(M, K, device=cuda, generator=gd) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=cuda, generator=gd) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    b = (torch.rand(N, device=cuda, generator=gd) - 0.5) if mode != "plain" else None
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


@pytest.mark.parametrize("M,N,K,S", [
    (8192, 768, 6272, 2),        # LM-head data gradient shape (K = 50,304 cut to 98 K-tiles for test time)
    (1000, 520, 4096, 3),        # M / N tails, ragged last split (64 K-tiles / 3)
    (256, 256, 64 * 9, 4),       # 9 K-tiles in 4 splits (the last one short)
    (512, 1032, 2048, 16),       # N % 256 != 0, many splits
])
def test_gemm_pp_splitk_matches_fp32(cuda, M, N, K, S):
    """Split-K (EPI 6 partial slabs + the ordered reduction): forced split
    counts against the fp32 reference, and the split result equal to the
    unsplit kernel to fp32-summation-order rounding of the bf16 output."""
    from distributed_compute_pytorch_amd._ext import C

    g = torch.Generator(device=cuda).manual_seed(5)
    x = (torch.rand(M, K, device=cuda, generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=cuda, generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    ref = _ref(x, w, None)
    old = (C.gemm_tune_get("pp_sk"), C.gemm_tune_get("pp_sk_force"))
    try:
        C.gemm_tune("pp_sk_force", S)
        y = C.gemm_pp(x, w)[0]
        C.gemm_tune("pp_sk_force", 0)
        C.gemm_tune("pp_sk", 0)
        y1 = C.gemm_pp(x, w)[0]
    finally:
        C.gemm_tune("pp_sk", old[0])
        C.gemm_tune("pp_sk_force", old[1])
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 6e-3
    assert _rel(y, y1) < 6e-3
    # repeatable: the reduction order is fixed
    C.gemm_tune("pp_sk_force", S)
    try:
        y2 = C.gemm_pp(x, w)[0]
    finally:
        C.gemm_tune("pp_sk_force", old[1])
    assert torch.equal(y, y2)


def test_gemm_pp_splitk_plan():
    """The split count the time model picks: the LM-head data gradient (96
    tiles, 786 K-tiles) splits; full-chip shapes and short K do not."""
    from distributed_compute_pytorch_amd._ext import C

    assert C.gemm_pp_splitk(8192, 768, 50304) >= 2
    assert C.gemm_pp_splitk(8192, 2304, 768) == 1
    assert C.gemm_pp_splitk(8192, 768, 768) == 1
