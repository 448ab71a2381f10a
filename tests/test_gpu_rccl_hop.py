"""RCCL communicator multi-rank code path, exercised on one GPU.

DCP_SINGLE_RANK_HOP=1 forces the 1-rank communicator through the comm-stream
hop with real RCCL calls (see tests/gpu_hop_worker.py): stream ordering of
producer -> collective -> consumer, every collective, DDP through the comm
stream (fp32 / bf16 wire / bucket views, with no_sync) against local training,
and the find_unused_parameters device used-map.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_single_rank_hop_real_rccl(cuda):
    env = dict(os.environ, DCP_SINGLE_RANK_HOP="1", DCP_COMM_TIMING="1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_hop_worker.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("HOPRESULT ")][-1]
    res = json.loads(line[len("HOPRESULT "):])
    print(res)
    assert res["comm_stream"] and res["comm_stream_differs"]
    assert res["ordering_ok"]
    assert res["reduce_into_ok"]
    assert res["collectives_ok"]
    assert res["ops_issued"] >= 8
    errs = res["ddp_max_abs_err"]
    assert errs["fp32"] < 1e-5, errs
    assert errs["grad_view"] < 1e-5, errs
    assert errs["bf16_wire"] < 5e-2, errs  # bf16 gradients on the wire
    assert errs["bf16_hook"] < 5e-2, errs  # the same through bf16_compress_hook (async cast back)
    assert errs["overlap"] < 1e-5, errs  # optimizer synced bucket by bucket (overlap_optimizer)
    assert errs["overlap_sliced"] < 1e-5, errs  # oversize bucket as slice collectives (bucket_slice_mb)
    assert errs["overlap_sliced_adam"] < 1e-4, errs  # fused AdamW on the slices' parameter ranges
    assert errs["fp32_buckets"] >= 2
    assert errs["registered"] < 1e-5, errs  # bucket buffers registered with ncclCommRegister
    assert res["register_handle"] > 0 and res["registered_allreduce_ok"]
    assert res["unused_ok"] and res["globally_unused_grad_none"]


def test_single_rank_hop_with_stream_ordering_check(cuda):
    """Same worker with the Reducer's debug stream-ordering check on
    (DCP_DEBUG_STREAMS=1): every bucket's pack -> RCCL collective (comm stream)
    -> consumer edge is verified by checksum; any violation raises in finalize."""
    env = dict(os.environ, DCP_SINGLE_RANK_HOP="1", DCP_DEBUG_STREAMS="1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "gpu_hop_worker.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "stream-ordering check failed" not in r.stderr
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("HOPRESULT ")][-1]
    res = json.loads(line[len("HOPRESULT "):])
    assert res["ordering_ok"] and res["collectives_ok"]
    assert res["ddp_max_abs_err"]["fp32"] < 1e-5
