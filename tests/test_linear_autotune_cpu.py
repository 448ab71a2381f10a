"""Linear GEMM selection (ops/linear.py): pinned choices round-trip through a
JSON table and win over measuring; with autotune off the default kernel runs
(what the GPU numerics tests rely on to validate our kernels, not hipBLASLt)."""
import json

from distributed_compute_pytorch_amd.ops import linear as lin


def _cands(log):
    return {n: (lambda n=n: log.append(n)) for n in ("pp", "ring", "hipblaslt")}


def test_default_when_autotune_off(monkeypatch):
    monkeypatch.setattr(lin, "_AUTOTUNE", False)
    monkeypatch.setattr(lin, "_CHOICE", {})
    for d in ("pp", "ring"):
        monkeypatch.setattr(lin, "_DEFAULT_OURS", d)
        assert lin._pick(("fwd", 8, 64, 64), _cands([])) == d
    # a shape the ping-pong GEMM does not take falls back to the ring
    monkeypatch.setattr(lin, "_DEFAULT_OURS", "pp")
    c = _cands([])
    del c["pp"]
    assert lin._pick(("fwd", 8, 64, 60), c) == "ring"
    assert lin._CHOICE == {}  # nothing measured, nothing recorded


def test_pinned_choices_roundtrip(monkeypatch, tmp_path):
    monkeypatch.setattr(lin, "_CHOICE", {("fwd", 8192, 768, 2304): "pp", ("dgrad", 8192, 2304, 768): "hipblaslt"})
    path = tmp_path / "choices.json"
    lin.save_choices(str(path))
    table = json.loads(path.read_text())
    assert table == {"fwd 8192 768 2304": "pp", "dgrad 8192 2304 768": "hipblaslt"}
    table["fwd_gelu 16 64 128"] = "ours"  # round-3 tables name the ring "ours"
    path.write_text(json.dumps(table))
    monkeypatch.setattr(lin, "_CHOICE", {})
    lin.load_choices(str(path))
    assert lin._CHOICE[("fwd_gelu", 16, 64, 128)] == "ring"
    # pinned choices win over measuring (which would need a GPU here)
    monkeypatch.setattr(lin, "_AUTOTUNE", True)
    assert lin._pick(("dgrad", 8192, 2304, 768), _cands([])) == "hipblaslt"


def test_agree_single_process_keeps_local_choice():
    assert lin._agree(("fwd", 1, 2, 3), "ring") == "ring"


def _agree_world(rank, world):
    import time

    from distributed_compute_pytorch_amd import distributed as dist

    lin._AGREE_WAIT_S = 0.5
    mine = "pp" if rank == 0 else "ring"
    # a shape every rank runs: rank 0's measurement wins everywhere
    assert lin._agree(("fwd", 64, 64, 64), mine) == "pp"
    # a shape only rank 1 runs (uneven last batch, rank-dependent path): rank 1
    # keeps its own choice after a bounded wait instead of blocking on rank 0
    if rank == 1:
        t0 = time.time()
        assert lin._agree(("fwd", 63, 64, 64), "hipblaslt") == "hipblaslt"
        assert time.time() - t0 < 10
    dist.barrier()


def test_agree_takes_rank0_choice_and_never_blocks():
    from mp_util import run_world

    run_world(_agree_world, 2)


def test_near_ties_go_to_our_kernels(monkeypatch):
    monkeypatch.setattr(lin, "_AUTOTUNE", True)
    monkeypatch.setattr(lin, "_CHOICE", {})
    times = {}
    monkeypatch.setattr(lin, "_measure", lambda cands: dict(times))
    monkeypatch.setattr(lin.torch.cuda, "is_current_stream_capturing", lambda: False)  # no GPU here
    assert lin._OURS_TIE == 0.12  # the default band (sustained-load bias, NOTES §33)
    times.update(pp=1.10, ring=1.2, hipblaslt=1.0)  # within 12 %: ours
    assert lin._pick(("fwd", 1, 2, 3), _cands([])) == "pp"
    times.update(pp=1.15, ring=1.14, hipblaslt=1.0)  # 14 % slower: hipBLASLt
    assert lin._pick(("fwd", 1, 2, 4), _cands([])) == "hipblaslt"
    times.update(pp=0.9, ring=1.2, hipblaslt=1.0)
    assert lin._pick(("fwd", 1, 2, 5), _cands([])) == "pp"


def _pretune_world(rank, world):
    """ops.linear.pretune: inside, every rank decides each shape from its own
    measurement (no per-shape store key, no wait); on exit rank 0's table is
    adopted by every rank in one store round — shapes only this rank met keep
    the local choice."""
    from distributed_compute_pytorch_amd import distributed as dist

    lin._CHOICE.clear()
    lin._AUTOTUNE = True
    fastest = "pp" if rank == 0 else "ring"
    # a fake measurement: this rank's favourite wins by 30 %
    lin._measure = lambda cands, rounds=3: {k: (1.0 if k == fastest else 1.3) for k in cands}
    import torch

    torch.cuda.is_current_stream_capturing = lambda: False  # (no device in this process)
    with lin.pretune():
        assert lin._pick(("fwd", 64, 64, 64), _cands([])) == fastest
        assert lin._pick(("dgrad", 64, 64, 64), _cands([])) == fastest
        if rank == 1:
            assert lin._pick(("fwd", 32, 64, 64), _cands([])) == "ring"
    pg = dist.get_default_group()
    assert not pg.store.check(["dcp/linear_autotune/fwd 64 64 64"])  # no per-shape agreement ran
    assert lin._CHOICE[("fwd", 64, 64, 64)] == "pp"
    assert lin._CHOICE[("dgrad", 64, 64, 64)] == "pp"
    if rank == 1:
        assert lin._CHOICE[("fwd", 32, 64, 64)] == "ring"
    # later steps find the shapes decided: _pick returns without measuring
    lin._measure = None
    assert lin._pick(("fwd", 64, 64, 64), _cands([])) == "pp"


def test_pretune_table_adopted_from_rank0():
    from mp_util import run_world

    run_world(_pretune_world, 2)


def test_pp_xent_choice_pins_and_roundtrips(monkeypatch, tmp_path):
    """The LM head's fused GEMM + loss partials ("pp_xent") is a valid choice
    for pinned tables (and so for the rank-0 table every rank adopts)."""
    monkeypatch.setattr(lin, "_CHOICE", {})
    path = tmp_path / "pin.json"
    path.write_text(json.dumps({"head_xent 8192 768 50304": "pp_xent"}))
    lin.load_choices(str(path))
    assert lin._CHOICE == {("head_xent", 8192, 768, 50304): "pp_xent"}
    log = []
    cands = {n: (lambda n=n: log.append(n)) for n in ("pp_xent", "pp", "hipblaslt")}
    assert lin._pick(("head_xent", 8192, 768, 50304), cands) == "pp_xent" and log == []
