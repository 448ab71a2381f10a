"""Weight gradient on the 8-wave ping-pong kernel (csrc/kernels/wgrad_pp.hip)
against fp64 references of the same op (bf16 operands are exact in fp64, so
the only error left is the kernel's fp32 accumulation): Linear / 1x1 shapes
(one slab written straight into D, several slabs + the ordered reduction,
ragged row counts, channel counts past the last full 256-wide tile, the
padded-vocabulary ``out_rows`` head, accumulation into an existing gradient)
and the gathered kxk convolution wgrad (stride 1 / 2, zero padding)."""
import contextlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@contextlib.contextmanager
def _tune(**kv):
    from distributed_compute_pytorch_amd._ext import C as _C

    old = {k: _C.gemm_tune_get(k) for k in kv}
    try:
        for k, v in kv.items():
            _C.gemm_tune(k, v)
        yield
    finally:
        for k, v in old.items():
            _C.gemm_tune(k, v)


def _bf(shape, gen, dev):
    return torch.randn(*shape, generator=gen).to(torch.bfloat16).to(dev)


LINEAR = [  # (M, N1 = out features, N2 = in features)
    (8192, 768, 3072),   # GPT-2 fc2 wgrad: several slabs
    (8192, 3072, 768),   # GPT-2 fc
    (16384, 2304, 768),  # BERT qkv
    (512, 512, 256),     # 8 K-tiles: one slab, straight into D
    (1000, 256, 320),    # ragged last K-tile; N2 past the last full tile
    (3000, 320, 512),    # N1 past the last full tile, several slabs
]


@pytest.mark.parametrize("shape", LINEAR)
def test_wgrad_pp_linear(cuda, shape):
    from distributed_compute_pytorch_amd._ext import C as _C

    m, n1, n2 = shape
    g = torch.Generator().manual_seed(11)
    gy, x = _bf((m, n1), g, cuda), _bf((m, n2), g, cuda)
    ref = gy.double().t() @ x.double()
    with _tune(wg_pp=1):
        dw = _C.conv1x1_wgrad(gy, x)
    assert dw.dtype == torch.float32 and dw.shape == (n1, n2)
    assert _rel(dw, ref) < 1e-5
    with _tune(wg_pp=0):  # the ring kernel: same result to fp32 rounding
        dw0 = _C.conv1x1_wgrad(gy, x)
    assert _rel(dw0, ref) < 1e-5


@pytest.mark.parametrize("m", [2048, 16384])  # one slab (in-kernel +=) / several (+= in the reduction)
def test_wgrad_pp_accumulate_out_rows(cuda, m):
    """The padded-vocabulary head: N1 = 2,112 rows of which 2,100 exist in
    the gradient, accumulated into it (gradient-accumulation micro-steps)."""
    from distributed_compute_pytorch_amd._ext import C as _C

    n1, n2, rows = 2112, 768, 2100
    g = torch.Generator().manual_seed(12)
    gy, x = _bf((m, n1), g, cuda), _bf((m, n2), g, cuda)
    gy[:, rows:] = 0  # the pad columns carry no gradient (as in ops/lm_head.py)
    base = torch.randn(rows, n2, generator=g).to(cuda)
    acc = base.clone()
    with _tune(wg_pp=1):
        out = _C.conv1x1_wgrad(gy, x, accumulate_into=acc, out_rows=rows)
    assert out.data_ptr() == acc.data_ptr()
    ref = base.double() + (gy.double().t() @ x.double())[:rows]
    assert _rel(acc, ref) < 1e-5
    fresh = _C.conv1x1_wgrad(gy, x, out_rows=rows)
    assert fresh.shape == (rows, n2)
    assert _rel(fresh, (gy.double().t() @ x.double())[:rows]) < 1e-5


def test_wgrad_pp_slab_plans_agree(cuda):
    """Different split-over-rows plans give the same sums to fp32 rounding
    (slab count 1, several, and more than the reduction's 16-slab group)."""
    from distributed_compute_pytorch_amd._ext import C as _C

    m, n1, n2 = 8192, 512, 512
    g = torch.Generator().manual_seed(13)
    gy, x = _bf((m, n1), g, cuda), _bf((m, n2), g, cuda)
    ref = gy.double().t() @ x.double()
    for slots, min_kt in ((4, 128), (64, 4), (512, 1)):
        with _tune(wg_pp=1, wgpp_slots=slots, wgpp_min_kt=min_kt):
            dw = _C.conv1x1_wgrad(gy, x)
        assert _rel(dw, ref) < 1e-5, (slots, min_kt)


def _conv_wgrad_ref(gy, x, k, s, p):
    """dW[co, ci, kh, kw] in fp64 by unfold (no fp64 convolution kernel needed)."""
    n, co, ho, wo = gy.shape
    cols = F.unfold(x.double(), k, padding=p, stride=s)  # [n, ci*k*k, L]
    dw = torch.einsum("ncl,nkl->ck", gy.double().reshape(n, co, ho * wo), cols)
    return dw.reshape(co, x.shape[1], k, k)


@pytest.mark.parametrize("shape", [  # (N, H, W, Cin, Cout, k, stride, pad)
    (8, 14, 14, 256, 256, 3, 1, 1),   # ResNet layer 3
    (4, 14, 14, 256, 256, 3, 2, 1),   # layer-3 entry (stride 2)
    (8, 7, 7, 512, 512, 3, 1, 1),     # layer 4
    (2, 9, 11, 256, 320, 3, 1, 1),    # ragged rows, Cout past the last full tile
    (3, 12, 10, 320, 256, 3, 2, 1),   # Cin past the last full tile, stride 2, odd geometry
])
def test_wgrad_pp_conv_gathered(cuda, shape):
    from distributed_compute_pytorch_amd._ext import C as _C

    n, h, w, ci, co, k, s, p = shape
    g = torch.Generator().manual_seed(14)
    x = torch.randn(n, ci, h, w, generator=g).to(torch.bfloat16).to(cuda).contiguous(memory_format=torch.channels_last)
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    gy = torch.randn(n, co, ho, wo, generator=g).to(torch.bfloat16).to(cuda).contiguous(
        memory_format=torch.channels_last)
    ref = _conv_wgrad_ref(gy, x, k, s, p)
    with _tune(wg_pp=1):
        dw = _C.conv_wgrad(gy, x, k, k, s, p)
    assert dw.shape == ref.shape and dw.dtype == torch.float32
    assert _rel(dw, ref) < 1e-5
    with _tune(wg_pp=0):
        dw0 = _C.conv_wgrad(gy, x, k, k, s, p)
    assert _rel(dw0, ref) < 1e-5


def test_wgrad_pp_tail_split(cuda):
    """Tail split (wgrad_pp_plan): whole tiles straight into D, the last,
    partial round's tiles split over rows into slabs that the reduction adds
    from wgrad_pp_tail_row0 on — forced at small sizes by a small slot count.
    Linear with the padded-vocabulary out_rows + accumulation, a gathered 3x3
    conv (taps in the workgroup count) and a two-segment launch."""
    from distributed_compute_pytorch_amd._ext import C as _C

    g = torch.Generator().manual_seed(15)
    # 9 x 3 = 27 tiles on 24 slots: 24 whole, the last band of 3 in 8 slabs
    m, n1, n2, rows = 4096, 2112, 768, 2100
    gy, x = _bf((m, n1), g, cuda), _bf((m, n2), g, cuda)
    gy[:, rows:] = 0
    full = (gy.double().t() @ x.double())
    base = torch.randn(rows, n2, generator=g).to(cuda)
    for tail in (1, 0):
        with _tune(wg_pp=1, wgpp_slots=24, wgpp_min_kt=8, wgpp_tail=tail):
            acc = base.clone()
            _C.conv1x1_wgrad(gy, x, accumulate_into=acc, out_rows=rows)
            dw = _C.conv1x1_wgrad(gy, x)
        assert _rel(acc, base.double() + full[:rows]) < 1e-5, tail
        assert _rel(dw, full) < 1e-5, tail
    # 3 tiles x 9 taps = 27 workgroups on 24 slots: 2 tiles whole, 1 in 2 slabs
    x4 = torch.randn(4, 256, 14, 14, generator=g).to(torch.bfloat16).to(cuda).contiguous(
        memory_format=torch.channels_last)
    gy4 = torch.randn(4, 768, 14, 14, generator=g).to(torch.bfloat16).to(cuda).contiguous(
        memory_format=torch.channels_last)
    with _tune(wg_pp=1, wgpp_slots=24, wgpp_min_kt=1):
        dw = _C.conv_wgrad(gy4, x4, 3, 3, 1, 1)
    assert _rel(dw, _conv_wgrad_ref(gy4, x4, 3, 1, 1)) < 1e-5
    # two segments (micro-steps) in one launch under the tail plan
    gys = [_bf((r, n1), g, cuda) for r in (2048, 2000)]
    xs = [_bf((r, n2), g, cuda) for r in (2048, 2000)]
    ref = sum(a.double().t() @ b.double() for a, b in zip(gys, xs))
    with _tune(wg_pp=1, wgpp_slots=24, wgpp_min_kt=8):
        dw = _C.conv1x1_wgrad_multi(gys, xs)
    assert _rel(dw, ref) < 1e-5
