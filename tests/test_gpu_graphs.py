"""Whole-step HIP-graph capture: replays must equal eager execution."""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_captured_step_matches_eager(cuda):
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port
    from distributed_compute_pytorch_amd.models import resnet18_like
    from distributed_compute_pytorch_amd.utils.graphs import CapturedStep, capture_stream

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    try:
        torch.manual_seed(0)
        base = resnet18_like(num_classes=10, fused_bn=True).to(cuda).to(memory_format=torch.channels_last)
        m_eager, m_graph = copy.deepcopy(base), copy.deepcopy(base)
        d_e = dcp.parallel.DistributedDataParallel(m_eager, device_ids=[0], gradient_as_bucket_view=True)
        s = capture_stream()
        with torch.cuda.stream(s):
            d_g = dcp.parallel.DistributedDataParallel(m_graph, device_ids=[0], gradient_as_bucket_view=True)
        # small LR: a diverging run amplifies the (atomic-order) run-to-run
        # noise of the BN reductions into O(1) loss differences
        o_e = dcp.optim.SGD(d_e.parameters(), lr=0.005, momentum=0.9)
        o_g = dcp.optim.SGD(d_g.parameters(), lr=0.005, momentum=0.9)
        g = torch.Generator(device="cpu").manual_seed(1)
        batches = [(torch.randn(8, 3, 64, 64, generator=g).to(cuda).contiguous(memory_format=torch.channels_last),
                    torch.randint(0, 10, (8,), generator=g).to(cuda)) for _ in range(8)]

        def make(ddp, opt):
            def run(x, y):
                opt.zero_grad(set_to_none=True)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = F.cross_entropy(ddp(x), y)
                loss.backward()
                opt.step()
                return loss
            return run

        run_e, run_g = make(d_e, o_e), make(d_g, o_g)
        # the capture helper runs 3 warmup steps on the first batch
        for _ in range(3):
            run_e(*batches[0])
        cap = CapturedStep(run_g, [t.clone() for t in batches[0]], warmup=3, stream=s)  # capture does not execute

        def sync_state():
            # start every compared step from identical state (in place: the
            # graph keeps its addresses); chaotic drift of two independent
            # runs (MIOpen / atomic-order noise) is not what this test checks
            with torch.no_grad():
                for a, b in zip(m_eager.state_dict().values(), m_graph.state_dict().values()):
                    b.copy_(a)
                for pe, pg in zip(m_eager.parameters(), m_graph.parameters()):
                    o_g.state[pg]["momentum_buffer"].copy_(o_e.state[pe]["momentum_buffer"])

        for b in batches[1:5]:
            sync_state()
            torch.cuda.synchronize()
            le = run_e(*b).item()
            lg = cap(*b).item()
            torch.cuda.synchronize()
            assert abs(le - lg) < 1e-2 * max(1.0, abs(le)), (le, lg)
            for p, q in zip(m_eager.parameters(), m_graph.parameters()):
                rel = float((p - q).norm() / p.norm().clamp_min(1e-12))
                assert rel < 1e-3, rel
    finally:
        dcp.distributed.destroy_process_group()


def test_dropout_masks_fresh_per_replay(cuda):
    """The captured dropout reads the device Philox counter: each replay draws a
    new mask, and the captured backward regenerates the same mask."""
    from distributed_compute_pytorch_amd.ops import fused_dropout

    x = torch.randn(4096, device=cuda, requires_grad=True)
    fused_dropout(x, 0.5).sum().backward()  # eager warmup (creates the counter)
    x.grad = None
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y = fused_dropout(x, 0.5)
        y.sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    x.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        y = fused_dropout(x, 0.5)
        y.sum().backward()
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        m = y.detach() != 0
        assert torch.equal(x.grad != 0, m)
        masks.append(m.clone())
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])
