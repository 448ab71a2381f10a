"""Worker for tests/test_gpu_rccl_hop.py (run in a fresh process: the
communicator reads DCP_SINGLE_RANK_HOP at construction).

With DCP_SINGLE_RANK_HOP=1 a 1-rank RCCL communicator takes the multi-rank
path: every collective is a real ncclAllReduce / ncclBroadcast / ... call on
the dedicated comm stream, ordered after the caller's stream by an event, and
Work.wait() orders the caller after it. Checks:

* producer -> collective -> consumer ordering: the producer is a long spin
  kernel followed by a fill on the compute stream; an out-of-place all_gather
  (observable even on one rank) must see the fill, and a consumer after
  wait() must see the gathered values;
* every collective of the API returns the 1-rank identity;
* DDP (Reducer buckets on the comm stream) == local training, with no_sync
  accumulation and bf16 wire compression;
* find_unused_parameters through the device used-map path.
Prints one JSON line with the results.
"""
import json
import os
import sys

import torch
import torch.nn.functional as F
from torch import nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import distributed_compute_pytorch_amd as dcp
    from distributed_compute_pytorch_amd.distributed.launch import free_port
    from distributed_compute_pytorch_amd.models import ConvNet

    assert os.environ.get("DCP_SINGLE_RANK_HOP") == "1"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dcp.distributed.init_process_group("rccl", device_id=0)
    pg = dcp.distributed.get_default_group()
    comm = pg.rccl_comm()
    res = {"comm_stream": int(comm.stream_handle) != 0}
    cur = torch.cuda.current_stream().cuda_stream
    res["comm_stream_differs"] = int(comm.stream_handle) != int(cur)

    # ---- ordering: spin (~50 ms) -> fill -> all_gather (comm stream) -> consumer
    ok = True
    for trial in range(3):
        src = torch.zeros(1 << 20, device=dev)
        out = torch.full((1 << 20,), -1.0, device=dev)
        torch.cuda._sleep(50_000_000)
        src.fill_(float(trial + 1))
        w = comm.all_gather(out, src)
        w.wait()
        consumed = out * 2
        torch.cuda.synchronize()
        ok = ok and bool((consumed == 2.0 * (trial + 1)).all())
    res["ordering_ok"] = ok
    # all_reduce_into (compression hooks): the cast back is ordered before the Work
    ok = True
    for trial in range(3):
        wire = torch.zeros(1 << 20, device=dev, dtype=torch.bfloat16)
        out = torch.full((1 << 20,), -1.0, device=dev)
        torch.cuda._sleep(50_000_000)
        wire.fill_(float(trial + 1))
        w = comm.all_reduce_into(wire, out, dcp.distributed.ReduceOp.AVG)
        w.wait()
        consumed = out * 2
        torch.cuda.synchronize()
        ok = ok and bool((consumed == 2.0 * (trial + 1)).all())
    res["reduce_into_ok"] = ok

    # ---- every collective (identity on one rank)
    t = torch.arange(16, dtype=torch.float32, device=dev)
    ref = t.clone()
    dcp.distributed.all_reduce(t)
    dcp.distributed.all_reduce(t, dcp.distributed.ReduceOp.AVG)
    dcp.distributed.all_reduce(t, dcp.distributed.ReduceOp.MAX)
    dcp.distributed.broadcast(t, 0)
    g = torch.empty(16, device=dev)
    dcp.distributed.all_gather_into_tensor(g, t)
    rs = torch.empty(16, device=dev)
    dcp.distributed.reduce_scatter_tensor(rs, t)
    a2a = torch.empty(16, device=dev)
    dcp.distributed.all_to_all_single(a2a, t)
    dcp.distributed.barrier()
    torch.cuda.synchronize()
    res["collectives_ok"] = all(bool(torch.equal(x, ref)) for x in (t, g, rs, a2a))
    res["ops_issued"] = int(comm.ops_issued)

    # ---- DDP over the comm stream == local training (3 steps, accumulation 2)
    torch.manual_seed(0)
    base = ConvNet().to(dev)
    results = {}
    for name, kw in (("fp32", {}), ("bf16_wire", {"comm_dtype": torch.bfloat16}),
                     ("grad_view", {"gradient_as_bucket_view": True}),
                     ("registered", {"gradient_as_bucket_view": True, "register_buckets": True}),
                     ("bf16_hook", {"hook": dcp.parallel.comm_hooks.bf16_compress_hook}),
                     ("overlap", {"gradient_as_bucket_view": True, "overlap_optimizer": True}),
                     # fc1.weight (4.7 MB) reduced as 24 slice collectives
                     ("overlap_sliced", {"gradient_as_bucket_view": True, "overlap_optimizer": True,
                                         "bucket_slice_mb": 0.2}),
                     ("overlap_sliced_adam", {"gradient_as_bucket_view": True, "overlap_optimizer": True,
                                              "bucket_slice_mb": 0.2, "adam": True})):
        hook = kw.pop("hook", None)
        adam = kw.pop("adam", False)
        local = ConvNet().to(dev)
        local.load_state_dict(base.state_dict())
        mine = ConvNet().to(dev)
        mine.load_state_dict(base.state_dict())
        ddp = dcp.parallel.DistributedDataParallel(mine, device_ids=[0], bucket_cap_mb=1, **kw)
        if hook is not None:
            ddp.register_comm_hook(None, hook)
        local.eval(), mine.eval()
        if adam:  # the per-slice parameter-range updates
            o1 = torch.optim.AdamW(local.parameters(), lr=1e-3)
            o2 = dcp.optim.AdamW(ddp.parameters(), lr=1e-3)
        else:
            o1 = torch.optim.SGD(local.parameters(), lr=0.05, momentum=0.9)
            o2 = dcp.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
        gen = torch.Generator().manual_seed(3)
        for it in range(3):
            xs = [torch.randn(16, 1, 28, 28, generator=gen).to(dev) for _ in range(2)]
            ys = [torch.randint(0, 10, (16,), generator=gen).to(dev) for _ in range(2)]
            for m, o in ((local, o1), (ddp, o2)):
                o.zero_grad(set_to_none=True)
                for k in range(2):
                    ctx = ddp.no_sync() if (m is ddp and k == 0) else _Null()
                    with ctx, torch.enable_grad():
                        F.nll_loss(m(xs[k]), ys[k]).backward()
                o.step()
        err = max(float((p - q).abs().max()) for p, q in zip(local.parameters(), mine.parameters()))
        results[name] = err
        info = ddp.ddp_logging_data()
        results[name + "_buckets"] = info["num_buckets"]
        del ddp
    res["ddp_max_abs_err"] = results
    # explicit registration round trip on the communicator
    buf = torch.randn(1 << 20, device=dev)
    h = comm.register_buffer(buf)
    res["register_handle"] = int(h)
    want = buf.clone()
    dcp.distributed.all_reduce(buf, dcp.distributed.ReduceOp.SUM)  # on the registered buffer
    torch.cuda.synchronize()
    res["registered_allreduce_ok"] = bool(torch.equal(buf, want))
    comm.deregister_buffer(h)

    # ---- find_unused_parameters through the device used-map
    class Branchy(nn.Module):
        def __init__(self):
            super().__init__()
            self.a, self.b, self.h = nn.Linear(16, 16), nn.Linear(16, 16), nn.Linear(16, 4)

        def forward(self, x, use_b):
            y = torch.tanh(self.a(x))
            return self.h(self.b(y) if use_b else y)

    torch.manual_seed(1)
    m = Branchy().to(dev)
    ddp = dcp.parallel.DistributedDataParallel(m, device_ids=[0], find_unused_parameters=True)
    x = torch.randn(8, 16, device=dev)
    for use_b in (True, False, True):
        m.zero_grad(set_to_none=True)
        ddp(x, use_b).sum().backward()
    torch.cuda.synchronize()
    res["unused_ok"] = m.b.weight.grad is not None and m.a.weight.grad is not None
    m.zero_grad(set_to_none=True)
    ddp(x, False).sum().backward()
    torch.cuda.synchronize()
    res["globally_unused_grad_none"] = m.b.weight.grad is None
    dcp.distributed.destroy_process_group()
    print("HOPRESULT " + json.dumps(res), flush=True)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


if __name__ == "__main__":
    main()
