"""The Linear autotune's timing (``ops/linear.py:_measure``): candidates
alternate call by call with one event pair per call (NOTES §33: the chip's
clock drifts under sustained load, so per-candidate groups of back-to-back
calls were biased). Checks that every candidate is timed the same number of
times, that a candidate doing 4x the work measures slower, and that the
grouped (round-5) and spin-gap variants still return the same keys."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cands(dev):
    a = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    calls = {"small": 0, "big": 0}

    def small():
        calls["small"] += 1
        return a @ a

    def big():
        calls["big"] += 1
        return b @ b

    return {"small": small, "big": big}, calls


def test_interleaved_measure_orders_by_work(cuda, monkeypatch):
    from distributed_compute_pytorch_amd.ops import linear

    monkeypatch.setattr(linear, "_INTERLEAVE", True)
    monkeypatch.setattr(linear, "_SPIN_US", 0.0)
    cands, calls = _cands(cuda)
    ts = linear._measure(cands)
    assert set(ts) == {"small", "big"}
    assert calls["small"] == calls["big"] == 1 + 12  # warm + 4 * rounds
    assert 0 < ts["small"] < ts["big"]  # 8x the FLOPs


@pytest.mark.parametrize("mode", ["grouped", "spin"])
def test_measure_variants(cuda, monkeypatch, mode):
    from distributed_compute_pytorch_amd.ops import linear

    monkeypatch.setattr(linear, "_INTERLEAVE", mode != "grouped")
    monkeypatch.setattr(linear, "_SPIN_US", 200.0 if mode == "spin" else 0.0)
    monkeypatch.setattr(linear, "_SPIN_RATE", [])
    cands, _ = _cands(cuda)
    ts = linear._measure(cands)
    assert set(ts) == {"small", "big"} and 0 < ts["small"] < ts["big"]
