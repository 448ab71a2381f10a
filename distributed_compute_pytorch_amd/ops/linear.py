"""``nn.Linear`` for the bf16 transformer path with a leaner backward.

Under autocast a stock Linear costs, besides its three GEMMs, a bf16→fp32 cast
of the weight gradient and a generic ATen reduction (+ cast) for the bias
gradient — ~1/6 of the non-GEMM kernel time of BERT-base / GPT-2-small
(profiles/r1_*_prof22.txt). :class:`FusedLinear` (same parameters and
state_dict keys) computes

* Y = X Wᵀ + b on our MFMA GEMM (``gemm.hip`` gemm_nt) with the bias — and
  for ``forward_gelu`` the GELU — in the epilogue (``_C.linear_fwd``): the
  pre-activation h and gelu(h) leave the kernel together, no separate GELU pass,
* dX = dY W on the same kernel with a cached transposed bf16 weight,
* dW in fp32 straight from our split-M MFMA wgrad GEMM (the reduction over
  B·T rows is spread over the whole chip),
* db with the hand-written deterministic column-sum kernel (``colsum``, fp32).
Shapes the GEMM does not take (in/out features not multiples of 64, > 4096
inputs) fall back to ATen for the forward / data gradient.
"""
from __future__ import annotations

import os

import torch
from torch import nn
from torch.nn import functional as F
from torch.utils.weak import WeakIdKeyDictionary

from .._ext import C as _C

# forward_gelu: Linear + bias + GELU with the fused GELU kernels (False: FusedLinear + ATen GELU)
_FUSED_GELU = True
# forward / data-gradient GEMMs on our gemm_nt (False: hipBLASLt through ATen;
# bench.py --linear-path, for same-box A/Bs)
_OUR_FWD = True
_OUR_DGRAD = True
# per GEMM shape, the first call (eager, not under HIP-graph capture) times the
# candidate kernels and keeps the fastest — as cudnn.benchmark does for
# convolutions: "pp" = the 256 x 256 8-wave ping-pong GEMM (gemm_pp.hip),
# "ring" = the 128 x 128 ring (gemm.hip gemm_nt), "hipblaslt" = ATen.
# (profiles/r4_gemm_pp_bench_variants.jsonl, NOTES §25)
_AUTOTUNE = True
_CHOICE: dict = {}
# our kernel when nothing is measured (autotune off, or under graph capture)
_DEFAULT_OURS = "pp"
# MLP blocks as one node with the GELU backward in the second GEMM's epilogue
# (False: two FusedLinear nodes + the GELU-backward kernel; bench.py --linear-path ours-unfused-mlp)
_FUSED_MLP = True
# every name a _pick candidate dict can hold ("pp_xent": the LM head GEMM with
# the loss partials in its epilogue, ops/lm_head.py) — rank agreement and
# pinned tables accept only these
_CANDIDATES = ("pp", "ring", "hipblaslt", "pp_xent")


_TIMES: dict = {}  # key -> {candidate: ms} of the autotune measurement


def _time_ms(fn, iters: int = 5) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


# interleave the candidates call by call (False: the round-5 groups of 5
# back-to-back calls per candidate, kept for A/B: DCP_AUTOTUNE_GROUPED=1)
_INTERLEAVE = os.environ.get("DCP_AUTOTUNE_GROUPED", "0") != "1"
# µs of a one-wave spin kernel before each timed call (0: none); A/B knob
_SPIN_US = float(os.environ.get("DCP_AUTOTUNE_SPIN_US", "0"))
_SPIN_RATE: list = []  # spin cycles per µs, measured once


def _spin_cycles() -> int:
    if _SPIN_US <= 0:
        return 0
    if not _SPIN_RATE:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        torch.cuda._sleep(2_000_000)
        e.record()
        e.synchronize()
        _SPIN_RATE.append(2_000_000 / max(s.elapsed_time(e) * 1e3, 1.0))
    return int(_SPIN_US * _SPIN_RATE[0])


def _measure(cands: dict, rounds: int = 3) -> dict:
    """Per-call time of each candidate (ms). Candidates alternate CALL BY
    CALL, in a rotating order, each call timed by its own event pair; the
    result is the median over ``4 * rounds`` calls. Inside a training step
    the chip's clock swings with power: the same 0.7 ms kernel measured
    588-900 µs over consecutive calls with nothing else running (rocprofv3
    trace, profiles/r6_autotune_clock_trace.txt), so groups of back-to-back
    calls per candidate timed whichever candidate landed in a dip as slower
    (the LM-head weight gradient: ours 770 µs in the autotune, 600-640 µs in
    the steady step). Alternating calls see the same clock. A candidate's
    failure propagates: shapes a kernel cannot take are left out of
    ``cands`` up front (``_fwd_cands`` / ``_pp_ok``)."""
    for fn in cands.values():  # warm (first-launch setup) before timing
        fn()
    if not _INTERLEAVE:
        ts = {k: [] for k in cands}
        for _ in range(rounds):
            for k, fn in cands.items():
                ts[k].append(_time_ms(fn))
        return {k: min(v) for k, v in ts.items()}
    names = list(cands)
    ev = {k: [] for k in names}
    spin = _spin_cycles()
    for i in range(4 * rounds):
        for j in range(len(names)):
            k = names[(i + j) % len(names)]
            if spin:
                torch.cuda._sleep(spin)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            cands[k]()
            e.record()
            ev[k].append((s, e))
    # the last event on this stream, not a device-wide sync: a bucket
    # collective on the comm stream may be in flight (first synced backward)
    e.synchronize()
    out = {}
    for k, pairs in ev.items():
        t = sorted(s.elapsed_time(e) for s, e in pairs)
        out[k] = t[len(t) // 2]
    return out


def autotune_choices() -> dict:
    """{"fwd|fwd_gelu|dgrad M K N": "pp" | "ring" | "hipblaslt"} chosen so far."""
    return {" ".join(str(k) for k in key): v for key, v in _CHOICE.items()}


# how long a rank other than 0 waits for rank 0's choice of a shape
_AGREE_WAIT_S = 5.0
_FELL_BACK: list = []  # shapes this rank decided alone (warned once)


def _agree(key, mine: str) -> str:
    """Best-effort: every rank takes rank 0's choice for ``key`` when rank 0
    has published it within ``_AGREE_WAIT_S`` (each rank times on its own GPU
    and close shapes can time either way; with one choice every rank runs the
    same kernels, the same numerics). Never blocks longer: a shape rank 0 does
    not run, or reaches much later (uneven last batch, sequence bucketing,
    rank-dependent code), keeps this rank's own measurement. That is safe —
    a kernel choice only changes rounding; DDP averages the gradients, so the
    replicas stay identical. Through the rendezvous store, not a device
    collective: the first call of a shape may sit inside a backward whose
    bucket collectives are in flight."""
    from .. import distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return mine
    pg = dist.get_default_group()
    k = "dcp/linear_autotune/" + " ".join(str(x) for x in key)
    if pg.rank() == 0:
        pg.store.set(k, mine.encode())
        return mine
    try:
        pg.store.wait([k], int(_AGREE_WAIT_S * 1000))
    except (RuntimeError, TimeoutError):  # rank 0 has no entry (yet): keep the local measurement
        if not _FELL_BACK:
            import warnings

            warnings.warn(f"rank {pg.rank()}: no rank-0 GEMM choice for {' '.join(str(x) for x in key)} within "
                          f"{_AGREE_WAIT_S:.0f} s; using this rank's own measurement ({mine}). Ranks may now run "
                          "different kernels for this shape (rounding differs; DDP still averages identical "
                          "gradients). Tune before training (workloads.pretune_step / ops.linear.pretune) to "
                          "avoid this.", RuntimeWarning, stacklevel=3)
        _FELL_BACK.append(key)
        return mine
    theirs = bytes(pg.store.get(k)).decode()
    return theirs if theirs in _CANDIDATES else mine


# near-ties go to our kernels: hipBLASLt is taken only when it measured more
# than this fraction faster than our best candidate. 12 %: the autotune times
# back-to-back calls, a sustained-load regime in which our kernels lose 5-15 %
# more than hipBLASLt's (NOTES §33: the LM-head weight gradient measures 15 %
# behind yet ties in the step; BERT's 16,384-row forwards measure 2-10 % behind
# yet pinned to ours the step is +0.6 %). Same-box A/B of the band, 2 % vs
# 12 %: GPT-2 711.4 vs 712.8, BERT 1,798.5 vs 1,802.8 samples/s
# (profiles/r6_ours_tie_ab.jsonl). DCP_OURS_TIE overrides it.
_OURS_TIE = float(os.environ.get("DCP_OURS_TIE", "0.12"))


def _fastest(ts: dict) -> str:
    c = min(ts, key=ts.get)
    if c == "hipblaslt":
        ours = [k for k in ts if k != "hipblaslt"]
        if ours:
            o = min(ours, key=ts.get)
            if ts[o] <= ts[c] * (1.0 + _OURS_TIE):
                return o
    return c


_PRETUNE = [0]
_TABLE_ROUND = [0]


class pretune:
    """Context for a tuning micro-step run before training (e.g. under
    ``DistributedDataParallel.no_sync``, so no bucket collective is in flight):
    each shape first met inside is measured and chosen locally, without the
    per-shape rank agreement; on exit rank 0's whole table is published in ONE
    store round and every rank adopts it (:func:`agree_table`). The
    synchronised steps then find every shape decided — no autotune, and no
    store wait, inside a backward whose bucket reductions are running."""

    def __enter__(self):
        _PRETUNE[0] += 1
        return self

    def __exit__(self, *exc):
        _PRETUNE[0] -= 1
        if exc[0] is None and _PRETUNE[0] == 0:
            agree_table()
        return False


def agree_table(timeout_s: float = 300.0) -> int:
    """Every rank adopts rank 0's choice for each shape rank 0 has decided
    (one blocking store round; the table is small). Shapes only this rank
    decided keep its own choice. Returns the number of choices changed here."""
    import json

    from .. import distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return 0
    pg = dist.get_default_group()
    _TABLE_ROUND[0] += 1
    k = f"dcp/linear_autotune_table/{_TABLE_ROUND[0]}"
    if pg.rank() == 0:
        pg.store.set(k, json.dumps(autotune_choices()).encode())
        return 0
    pg.store.wait([k], int(timeout_s * 1000))
    changed = 0
    for name, v in json.loads(bytes(pg.store.get(k)).decode()).items():
        kind, *dims = name.split()
        key = (kind, *(int(d) for d in dims))
        if v in _CANDIDATES and _CHOICE.get(key) != v:
            _CHOICE[key] = v
            changed += 1
    return changed


def _pick(key, cands: dict) -> str:
    """The kernel to run for ``key`` among ``cands`` (name -> zero-argument
    launch): the measured fastest (rank 0's measurement when a process group is
    up; a pinned table from ``DCP_LINEAR_CHOICES`` / :func:`load_choices` wins
    over measuring); ``_DEFAULT_OURS`` (else "ring") with autotune off."""
    c = _CHOICE.get(key)
    if c is not None and c in cands:
        return c
    if not _AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return _DEFAULT_OURS if _DEFAULT_OURS in cands else ("ring" if "ring" in cands else next(iter(cands)))
    with torch.no_grad():
        ts = _measure(cands)
    _TIMES[key] = ts
    c = _CHOICE[key] = _fastest(ts) if _PRETUNE[0] else _agree(key, _fastest(ts))
    return c


def save_choices(path: str) -> None:
    """Write the per-shape choices made so far (JSON, :func:`autotune_choices`
    form) so a later run can pin them and be reproduced kernel for kernel."""
    import json

    with open(path, "w") as f:
        json.dump(autotune_choices(), f, indent=1, sort_keys=True)


def load_choices(path: str) -> None:
    """Pin per-shape choices from a :func:`save_choices` table ("ours" is read
    as "ring", the round-3 name); shapes it does not list are still measured."""
    import json

    with open(path) as f:
        table = json.load(f)
    for k, v in table.items():
        kind, *dims = k.split()
        v = "ring" if v == "ours" else v
        if v not in _CANDIDATES:
            raise ValueError(f"{path}: {k!r} -> {v!r} (want one of {_CANDIDATES})")
        _CHOICE[(kind, *(int(d) for d in dims))] = v


if os.environ.get("DCP_LINEAR_CHOICES"):
    load_choices(os.environ["DCP_LINEAR_CHOICES"])


def autotune_times() -> dict:
    """{"fwd|fwd_gelu|dgrad M K N": {candidate: µs}} of the autotune measurements."""
    return {" ".join(str(k) for k in key): {n: round(t * 1e3, 1) for n, t in v.items()} for key, v in _TIMES.items()}


def _pp_ok(M: int, N: int, K: int) -> bool:
    """Shapes the ping-pong GEMM takes (K % 64, N % 8; 32-bit operand offsets)."""
    return K % 64 == 0 and N % 8 == 0 and M > 0 and M * K < 2**31 and N * K < 2**31


def _pp_bias_ok(N: int) -> bool:
    """The ping-pong GEMM's bias epilogue: the one-tile kernel (gemm_tune
    "pp_v1" = 1, N % 8 == 0) takes any N; the persistent one stages the bias in
    LDS next to its 133,120-B ring (≤ 160 KiB: N ≤ 7,168)."""
    return (_C.gemm_tune_get("pp_v1") == 1 and N % 8 == 0) or N * 4 + 133120 <= 160 * 1024


# let the fused Adam/AdamW write the bf16 weight copies the forward GEMMs read
# (False: one cast launch per weight per forward; NOTES §15)
_SHADOWS = True

# > 0 while gradients accumulate locally (DistributedDataParallel.no_sync): the
# backward then adds dW / db straight into existing fp32 .grad tensors inside
# the wgrad / column-sum kernels and returns None for them, skipping autograd's
# separate AccumulateGrad add (one elementwise launch per parameter per
# micro-step: 3.8 ms of a GPT-2 accum-4 step, profiles/r1_gpt2_prof64.txt).
# A plain global, not thread-local: the backward runs on autograd's device
# threads. The synchronising micro-step adds in place too (see inplace_grad).
_ACCUM_IN_PLACE = [0]


class accumulate_grads_in_place:
    """Context manager used by ``DistributedDataParallel.no_sync``."""

    def __enter__(self):
        _ACCUM_IN_PLACE[0] += 1
        return self

    def __exit__(self, *exc):
        _ACCUM_IN_PLACE[0] -= 1
        return False


def accumulating() -> bool:
    """Sampled by each op's FORWARD into ``ctx.accum`` (like torch's no_sync,
    whose decision is taken in DDP's forward): where ``backward()`` is called
    does not matter."""
    return _ACCUM_IN_PLACE[0] > 0


def _engine_accumulates(p) -> bool:
    """True when the running backward will execute ``p``'s AccumulateGrad node,
    i.e. this graph task writes ``p.grad`` at all: ``loss.backward()`` does;
    ``torch.autograd.grad(loss, x)`` and ``backward(inputs=[x])`` without
    ``p`` do not (they must leave ``p.grad`` untouched and, for
    ``autograd.grad(loss, params)``, receive the gradient as a return value)."""
    from torch.autograd.graph import get_gradient_edge

    try:
        return bool(torch._C._will_engine_execute_node(get_gradient_edge(p).node))
    except RuntimeError:  # autograd.grad() with leaf inputs: gradients are returned, not accumulated
        return False


def inplace_grad(p, shape, accum: bool = False):
    """``p.grad`` when a backward may add its fp32 contribution straight into
    it and return None instead (skipping autograd's separate AccumulateGrad
    add — one elementwise launch per parameter per micro-step, 2.37 ms of a
    GPT-2 accum-4 step: profiles/r2_gpt2_kernel_stats_final.txt:11), else None.

    Only when the running graph task accumulates into ``p.grad`` anyway
    (``_engine_accumulates``: not under ``autograd.grad`` / ``backward(inputs=)``
    that exclude ``p``), and then

    * under ``no_sync`` (``accum``): whenever ``.grad`` holds a compatible
      fp32 buffer (DDP ignores the hooks of these micro-steps);
    * on any other backward only when nothing could observe the difference:
      no gradient graph is being built (``create_graph``), and no tensor hook
      or post-accumulate hook sits on the parameter. The AccumulateGrad node
      still runs (with an undefined gradient) after every producer of the
      parameter's gradient — tied weights included — so the DDP Reducer's
      post-hook on it (``reducer.cpp`` register_hooks) fires exactly once,
      after the in-place add, and finds the accumulated ``.grad``.
    """
    if p is None or not p.is_leaf:  # a packed (concatenated) weight: autograd splits its gradient
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != shape or g.requires_grad:
        return None
    if not accum and (torch.is_grad_enabled() or p._backward_hooks or getattr(p, "_post_accumulate_grad_hooks", None)):
        return None
    if not _engine_accumulates(p):
        return None
    return g


def _acc_target(ctx, p, shape):
    return inplace_grad(p, shape, getattr(ctx, "accum", False))


# ---- micro-step weight-gradient deferral -----------------------------------
# DistributedDataParallel(defer_accum_wgrad=True): inside no_sync the Linear
# weight gradients are not computed. Their operands (dY and the saved X) are
# kept, and the synchronising micro-step computes each weight gradient over
# the rows of ALL its micro-steps in one ping-pong wgrad launch
# (_C.conv1x1_wgrad_multi, up to 4 row segments per launch): one split-over-rows
# slab plan and one slab reduction per step instead of one per micro-step —
# at GPT-2's 8,192-row micro-steps the slab writes and reduction are ~25 % of
# each wgrad (profiles/r5_wgrad_dispatches*.txt). Costs the kept operands'
# memory (~7 GB for GPT-2-small accum 4; the GPU has 288 GB).
# Until then p.grad lacks the deferred contributions: flush_weight_grads()
# adds them, and every optimizer step (a global torch.optim step pre-hook,
# stock and fused optimizers alike) calls it first.
_DEFER = [0]
_PENDING: dict = {}  # id(first parameter of the group) -> _Pending
_PENDING_B: dict = {}  # id(bias) -> (bias, [dY segments]): bias gradients deferred the same way
_HOOKED = [False]
# ids of the parameters whose Linear ran in the current synchronising forward
# (their backward consumes the pending segments); see flush_unclaimed
_CLAIMED: set = set()
# DDPs with defer_accum_wgrad over more than one rank: a flush at the
# optimizer step (after the all-reduce) would add unreduced contributions
_MULTI_RANK_DEFER = [0]


def _claim(params) -> None:
    """Forward of a Linear outside no_sync deferral: its backward will take
    any pending segments of ``params`` into the synchronised gradient."""
    if (_PENDING or _PENDING_B) and not _DEFER[0]:
        for p in params:
            if p is not None:
                _CLAIMED.add(id(p))


class _Pending:
    __slots__ = ("params", "rows", "segs")

    def __init__(self, params, rows):
        self.params, self.rows, self.segs = params, rows, []


class defer_weight_grads:
    """Context manager used by ``DistributedDataParallel.no_sync`` when the
    DDP was built with ``defer_accum_wgrad=True``."""

    def __enter__(self):
        _DEFER[0] += 1
        _install_flush_hook()
        return self

    def __exit__(self, *exc):
        _DEFER[0] -= 1
        return False


def deferring() -> bool:
    """Sampled by the forward into ``ctx.defer`` (as ``accumulating``)."""
    return _DEFER[0] > 0


def pending_weight_grads() -> int:
    """Parameters (groups) whose gradient has deferred micro-step contributions."""
    return len(_PENDING) + len(_PENDING_B)


def _install_flush_hook():
    if not _HOOKED[0]:
        from torch.optim.optimizer import register_optimizer_step_pre_hook

        register_optimizer_step_pre_hook(lambda opt, args, kwargs: flush_weight_grads(_at_step=True))
        _install_zero_grad_discard()
        _HOOKED[0] = True


def _install_zero_grad_discard():
    """The deferred contributions belong to ``.grad`` and must go with it:
    stock ``torch.optim.Optimizer.zero_grad`` and ``torch.nn.Module.zero_grad``
    (which have no hooks) are wrapped to drop the stash of their parameters
    first, as this package's optimizers' zero_grad does — otherwise an
    accumulation round abandoned by a stock zero_grad would leak its stashed
    micro-steps into the next round's synchronised gradient.
    Installed once, by the first deferring no_sync."""
    import functools

    opt_zg, mod_zg = torch.optim.Optimizer.zero_grad, torch.nn.Module.zero_grad

    @functools.wraps(opt_zg)
    def optimizer_zero_grad(self, *args, **kwargs):
        if _PENDING or _PENDING_B:
            discard_weight_grads([p for g in self.param_groups for p in g["params"]])
        return opt_zg(self, *args, **kwargs)

    @functools.wraps(mod_zg)
    def module_zero_grad(self, *args, **kwargs):
        if _PENDING or _PENDING_B:
            discard_weight_grads(list(self.parameters()))
        return mod_zg(self, *args, **kwargs)

    torch.optim.Optimizer.zero_grad = optimizer_zero_grad
    torch.nn.Module.zero_grad = module_zero_grad


def _wgrad_sum(segs, tgt):
    """Σ over the (gy, x) row segments, ≤ 4 per launch, into ``tgt`` (the
    existing fp32 gradient) when given, else a new fp32 tensor."""
    dw = tgt
    for i in range(0, len(segs), 4):
        chunk = segs[i:i + 4]
        dw = _C.conv1x1_wgrad_multi([g for g, _ in chunk], [x for _, x in chunk], accumulate_into=dw)
    return dw


def _colsum_sum(segs, tgt):
    """Σ of the rows of the dY segments, ≤ 4 per launch, into ``tgt`` when given."""
    db = tgt
    for i in range(0, len(segs), 4):
        db = _C.colsum_multi(segs[i:i + 4], accumulate_into=db)
    return db


def _flush_bias(b, segs) -> None:
    db = _colsum_sum(segs, None)
    with torch.no_grad():
        db = db.view(b.shape).to(b.dtype)
        if b.grad is None:
            b.grad = db
        else:
            b.grad.add_(db)


def _flush_weight(e) -> None:
    dw = _wgrad_sum(e.segs, None)
    parts = dw.split(e.rows, 0) if e.rows else (dw,)
    with torch.no_grad():
        for p, d in zip(e.params, parts):
            d = d.view(p.shape).to(p.dtype)
            if p.grad is None:
                p.grad = d
            else:
                p.grad.add_(d)


def flush_weight_grads(_at_step: bool = False) -> None:
    """Add every deferred micro-step weight / bias gradient into its
    parameters' ``.grad`` (creating it where None). Called by every optimizer
    step."""
    if _at_step and (_PENDING or _PENDING_B) and _MULTI_RANK_DEFER[0]:
        import warnings

        warnings.warn("deferred micro-step weight gradients flushed at the optimizer step, after the DDP "
                      "all-reduce: these contributions are local to this rank (was a no_sync accumulation "
                      "round not closed by a synchronised backward through the same Linears?)",
                      RuntimeWarning, stacklevel=3)
    while _PENDING_B:
        _flush_bias(*_PENDING_B.popitem()[1])
    while _PENDING:
        _flush_weight(_PENDING.popitem()[1])
    _CLAIMED.clear()


def flush_unclaimed(params=None) -> list:
    """After a synchronising forward: add into ``.grad`` — before the
    backward, so the bucket reductions cover them — the pending segments of
    every Linear (among ``params``; all when None) that did NOT run in that
    forward and so would never consume them. Torch DDP reduces the whole
    accumulated ``.grad``; without this, such contributions would reach
    ``.grad`` only at the optimizer step, unreduced (replicas diverge).
    Returns the parameters whose ``.grad`` received something."""
    done = []
    if not (_PENDING or _PENDING_B):
        _CLAIMED.clear()
        return done
    ids = None if params is None else {id(p) for p in params}
    for k in [k for k, e in _PENDING.items()
              if not any(id(p) in _CLAIMED for p in e.params) and (ids is None or id(e.params[0]) in ids)]:
        e = _PENDING.pop(k)
        _flush_weight(e)
        done.extend(e.params)
    for k in [k for k, (b, _) in _PENDING_B.items() if k not in _CLAIMED and (ids is None or k in ids)]:
        b, segs = _PENDING_B.pop(k)
        _flush_bias(b, segs)
        done.append(b)
    _CLAIMED.clear()
    return done


def discard_weight_grads(params=None) -> None:
    """Drop the deferred contributions — all of them, or those of ``params``
    (what a ``zero_grad`` of this package's optimizers clears: gradients
    stashed by no_sync micro-steps belong to ``.grad`` and go with it)."""
    if params is None:
        _PENDING.clear()
        _PENDING_B.clear()
        return
    ids = {id(p) for p in params}
    for k in [k for k, e in _PENDING.items() if all(id(p) in ids for p in e.params)]:
        del _PENDING[k]
    for k in [k for k, (b, _) in _PENDING_B.items() if id(b) in ids]:
        del _PENDING_B[k]


def _deferred_bias(ctx, bias, g2):
    """(handled, db) — the bias-gradient twin of _deferred_wgrad: under no_sync
    deferral keep dY (already kept for the weight gradient) instead of a
    column-sum launch per micro-step; the synchronising micro-step sums the
    rows of all of them in one launch (``_C.colsum_multi``)."""
    if (bias is None or not bias.is_leaf or not g2.is_cuda or g2.shape[1] % 8 != 0
            or not g2.is_contiguous()):
        return False, None
    key = id(bias)
    if getattr(ctx, "defer", False):
        if g2.shape[0] == 0 or not _engine_accumulates(bias):
            return False, None
        _PENDING_B.setdefault(key, (bias, []))[1].append(g2)
        return True, None
    e = _PENDING_B.pop(key, None)
    if e is None:
        return False, None
    tgt = _acc_target(ctx, bias, torch.Size((g2.shape[1],)))
    db = _colsum_sum(e[1] + ([g2] if g2.shape[0] else []), tgt)
    return True, (None if tgt is not None else db)


def _deferred_wgrad(ctx, g2, x2):
    """(handled, dw): stash (g2, x2) under no_sync deferral (handled, dw None),
    or — on the synchronising micro-step — dW over the stashed segments plus
    this one (returned, or added into the parameter's .grad: dw None)."""
    params = getattr(ctx, "defer_params", None)
    if params is None:
        w = ctx.params[0]
        params = (w,) if w is not None else None
    if params is None or not g2.is_cuda or not all(p.is_leaf for p in params):
        return False, None
    key = id(params[0])
    if getattr(ctx, "defer", False):
        if g2.shape[0] == 0 or not _engine_accumulates(params[0]):
            return False, None
        e = _PENDING.get(key)
        if e is None:
            e = _PENDING[key] = _Pending(params, getattr(ctx, "rows", None))
        e.segs.append((g2, x2.contiguous()))
        return True, None
    e = _PENDING.pop(key, None)
    if e is None:
        return False, None
    segs = e.segs + ([(g2, x2.contiguous())] if g2.shape[0] else [])  # (an empty micro-batch adds nothing)
    tgt = _acc_target(ctx, params[0], torch.Size((g2.shape[1], x2.shape[1]))) if len(params) == 1 else None
    dw = _wgrad_sum(segs, tgt)
    return True, (None if tgt is not None else dw)


def _gemm_ok(x: torch.Tensor, w: torch.Tensor, bias) -> bool:
    """Shapes our gemm_nt takes (in/out features multiples of 64, ≤ 4096 in)."""
    return (_OUR_FWD and bias is not None and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0 and w.shape[1] <= 4096
            and x.is_contiguous() and x.numel() > 0)


def _fwd_cands(x2, w, b, b32, mode: int) -> dict:
    """Forward candidates (Linear + bias [+ GELU: mode 1 tanh / 2 erf])."""
    M, K, N = x2.shape[0], w.shape[1], w.shape[0]
    c = {}
    if _pp_ok(M, N, K) and _pp_bias_ok(N):
        c["pp"] = lambda: _C.gemm_pp(x2, w, b32, mode)
    c["ring"] = lambda: _C.linear_fwd(x2, w, b32, mode)
    if mode:
        c["hipblaslt"] = lambda: _C.gelu_fwd(F.linear(x2, w, _lb(b)), mode == 1)
    else:
        c["hipblaslt"] = lambda: F.linear(x2, w, _lb(b))
    return c


def _wgrad_slots(M: int) -> int:
    """Workgroup budget of the split-M wgrad plan for an M-row Linear: twice
    the default (more, shorter M splits) from 16,384 rows — same-box A/B
    (profiles/r4_wgslots.jsonl): BERT (16,384 rows) 1,665 → 1,685 samples/s
    at 1,024, GPT-2 (8,192 rows) 621 → 614, so it keeps 512 (0 = default)."""
    return 1024 if M >= 16384 else 0


def _lb(b):
    """The bias as the bf16 ATen GEMMs take it, cast only where one runs (our
    kernels read the fp32 bias in their epilogue). A CUDA fp32 bias gets a
    registered bf16 shadow that the fused Adam/AdamW step rewrites with the
    update (as the weights' shadows): GPT-2's hipBLASLt MLP forward cast its
    biases 48 times a step otherwise."""
    if b is None or b.dtype == torch.bfloat16:
        return b
    if _SHADOWS and b.is_cuda and b.dtype == torch.float32 and not torch.cuda.is_current_stream_capturing():
        from ..optim.fused import fresh_bf16_shadow, register_bf16_shadow

        t = fresh_bf16_shadow(b)
        if t is None:
            t = b.detach().to(torch.bfloat16)
            register_bf16_shadow(b, t)
        return t
    return b.detach().to(torch.bfloat16)


def _bias32(bias: torch.Tensor) -> torch.Tensor:
    b = bias.detach()
    return b if b.dtype == torch.float32 and b.is_contiguous() else b.float().contiguous()


def _linear_fwd(x, w, b, bias):
    """x·wᵀ + b on the kernel the per-shape autotune picked (bf16 x, w; ``b``
    the bias as given, ``bias`` its fp32 parameter for our epilogues)."""
    if _gemm_ok(x, w, bias):
        x2, b32 = x.reshape(-1, x.shape[-1]), _bias32(bias)
        M, K, N = x2.shape[0], w.shape[1], w.shape[0]
        c = _pick(("fwd", M, K, N), _fwd_cands(x2, w, b, b32, 0))
        if c == "pp":
            return _C.gemm_pp(x, w, b32, 0)[0]
        if c == "ring":
            return _C.linear_fwd(x, w, b32, 0)[0]
    return F.linear(x, w, _lb(b))


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, w16, b16, w16t):
        x, w, b = _setup(ctx, x, weight, bias, w16, b16)
        ctx.save_for_backward(x, w, w16t)
        return _linear_fwd(x, w, b, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w, wt = ctx.saved_tensors
        gy = gy.contiguous()
        if gy.dtype != torch.bfloat16:
            gy = gy.to(torch.bfloat16)
        return _linear_backward(ctx, gy.view(-1, gy.shape[-1]), x, w, wt=wt) + (None, None, None)


def _setup(ctx, x, weight, bias, w16, b16):
    w = w16 if w16 is not None else weight.to(torch.bfloat16)
    b = (b16 if b16 is not None else bias.detach()) if bias is not None else None  # cast by _lb where ATen runs
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    ctx.wdtype = weight.dtype
    ctx.accum = accumulating()
    ctx.defer = deferring()
    _claim((weight, bias))
    ctx.bdtype = bias.dtype if bias is not None else None
    ctx.params = (weight, bias)
    return x, w, b


def _dgrad_cands(g2, w, wt) -> dict:
    """Data-gradient candidates: dX = dY·W, as dY·(Wᵀ)ᵀ on our NT GEMMs."""
    c = {}
    if _pp_ok(g2.shape[0], wt.shape[0], g2.shape[1]):
        c["pp"] = lambda: _C.gemm_pp(g2, wt)
    c["ring"] = lambda: _C.conv1x1_dgrad(g2, wt)
    c["hipblaslt"] = lambda: g2 @ w
    return c


def _linear_backward(ctx, g2, x, w, db=None, db_done=False, wt=None):
    """(dx, dW, db) of y = x Wᵀ + b from the bf16 [M, N] output gradient g2.
    ``db_done``: the bias gradient was already produced by the caller (``db``,
    or added into ``bias.grad`` when ``db`` is None). ``wt``: bf16 Wᵀ [K, N]
    — the data gradient then runs on our GEMM."""
    x2 = x.reshape(-1, x.shape[-1])
    dx = dw = None
    if ctx.needs_input_grad[0]:
        c = "hipblaslt"
        if (_OUR_DGRAD and wt is not None and g2.shape[0] > 0 and g2.shape[1] % 64 == 0 and g2.shape[1] <= 4096
                and wt.shape[0] % 64 == 0):
            c = _pick(("dgrad", g2.shape[0], g2.shape[1], wt.shape[0]), _dgrad_cands(g2, w, wt))
        if c == "pp":
            dx = _C.gemm_pp(g2, wt)[0].view(x.shape)
        elif c == "ring":
            dx = _C.conv1x1_dgrad(g2, wt).view(x.shape)
        else:
            dx = (g2 @ w).view(x.shape)
    weight, bias = ctx.params
    if ctx.needs_input_grad[1]:
        done = False
        if g2.shape[1] % 64 == 0 and x2.shape[1] % 64 == 0:
            done, dw = _deferred_wgrad(ctx, g2, x2)
        if done:
            pass
        elif g2.shape[0] > 0 and g2.shape[1] % 64 == 0 and x2.shape[1] % 64 == 0:
            # our split-M MFMA wgrad GEMM (gemm.hip): faster than hipBLASLt at
            # every BERT / GPT-2 shape (profiles/r1_linear_wgrad_bench.log)
            tgt = _acc_target(ctx, weight, torch.Size((g2.shape[1], x2.shape[1])))
            dw = _C.conv1x1_wgrad(g2, x2.contiguous(), accumulate_into=tgt, slots=_wgrad_slots(g2.shape[0]))
            if tgt is not None:
                dw = None  # added into weight.grad by the kernel
        else:
            dw = torch.mm(g2.t(), x2, out_dtype=torch.float32)
        if dw is not None and dw.dtype != ctx.wdtype:
            dw = dw.to(ctx.wdtype)
    if not db_done and ctx.bdtype is not None and ctx.needs_input_grad[2]:
        done_b, db = _deferred_bias(ctx, bias, g2)
        tgt = None if done_b else _acc_target(ctx, bias, torch.Size((g2.shape[1],)))
        if done_b:
            pass
        elif g2.shape[0] == 0:  # empty batch: a zero bias gradient (no column-sum launch)
            db = torch.zeros(g2.shape[1], device=g2.device, dtype=torch.float32)
        else:
            db = _C.colsum(g2, accumulate_into=tgt)
            if tgt is not None:
                db = None
    if db is not None and db.dtype != ctx.bdtype:
        db = db.to(ctx.bdtype)
    return dx, dw, db


class _LinearGeluFn(torch.autograd.Function):
    """y = gelu(x Wᵀ + b). Forward: bf16 GEMM (+bias epilogue) then the GELU
    kernel (``gelu.hip``). Backward: one kernel computes gh = gy·gelu'(h) AND the
    bias gradient's column sums (no separate column-sum pass over gh), then the
    Linear's dX GEMM and MFMA wgrad."""

    @staticmethod
    def forward(ctx, x, weight, bias, w16, b16, w16t, tanh_approx):
        x, w, b = _setup(ctx, x, weight, bias, w16, b16)
        ctx.tanh = tanh_approx
        mode = 1 if tanh_approx else 2
        x2 = x.reshape(-1, x.shape[-1])
        c = "hipblaslt"
        if _gemm_ok(x, w, bias):
            b32 = _bias32(bias)
            c = _pick(("fwd_gelu", x2.shape[0], w.shape[1], w.shape[0]), _fwd_cands(x2, w, b, b32, mode))
        if c == "pp":
            y, h = _C.gemm_pp(x, w, b32, mode)  # h and gelu(h) from one GEMM epilogue
        elif c == "ring":
            y, h = _C.linear_fwd(x, w, b32, mode)
        else:
            h = F.linear(x, w, _lb(b))
            y = _C.gelu_fwd(h, tanh_approx)
        ctx.save_for_backward(x, w, h, w16t)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, h, wt = ctx.saved_tensors
        gy = gy.contiguous()
        if gy.dtype != torch.bfloat16:
            gy = gy.to(torch.bfloat16)
        bias = ctx.params[1]
        want_db = ctx.bdtype is not None and ctx.needs_input_grad[2]
        tgt = _acc_target(ctx, bias, torch.Size((h.shape[-1],))) if want_db else None
        gh, db = _C.gelu_bwd(gy, h, ctx.tanh, want_db, accumulate_into=tgt)
        if tgt is not None:
            db = None  # added into bias.grad by the kernel
        g2 = gh.view(-1, gh.shape[-1])
        return _linear_backward(ctx, g2, x, w, db=db, db_done=True, wt=wt) + (None, None, None, None)


class FusedLinear(nn.Linear):
    """``nn.Linear`` whose bf16 GPU forward/backward runs through :class:`_LinearFn`
    (fp32 weight/bias gradients without cast passes); plain ``nn.Linear``
    everywhere else (CPU, fp32 without autocast)."""

    def _bf16(self, p: torch.Tensor, slot: str):
        """bf16 copy of a parameter, reused while it is unchanged (autograd
        version, fused-optimizer epoch, storage): an accum-4 GPT-2 step casts
        each weight once instead of four times. Never cached while a HIP graph
        is being captured (the cast must be part of every replay)."""
        if torch.cuda.is_current_stream_capturing():
            return None
        from ..optim.fused import fresh_bf16_shadow, param_epoch, register_bf16_shadow

        key = (p._version, param_epoch(), p.data_ptr())
        c = self.__dict__.get(slot)
        if c is not None and c[0] == key:
            return c[1]
        t = fresh_bf16_shadow(p)  # rewritten by the fused Adam/AdamW step: no cast launch
        if t is None:
            t = p.detach().to(torch.bfloat16)
            if _SHADOWS:
                register_bf16_shadow(p, t)
        self.__dict__[slot] = (key, t)
        return t

    def _bf16t(self, w16: torch.Tensor) -> torch.Tensor:
        """bf16 Wᵀ [in, out] for the data-gradient GEMM, cached like ``_bf16``."""
        if torch.cuda.is_current_stream_capturing():
            return w16.t().contiguous()
        from ..optim.fused import param_epoch

        p = self.weight
        key = (p._version, param_epoch(), p.data_ptr(), w16.data_ptr())
        c = self.__dict__.get("_w16t_cache")
        if c is not None and c[0] == key:
            return c[1]
        t = w16.t().contiguous()
        self.__dict__["_w16t_cache"] = (key, t)
        return t

    def _fast(self, x: torch.Tensor) -> bool:
        return x.is_cuda and self.in_features % 8 == 0 and self.out_features % 8 == 0 and (
            x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                          and torch.get_autocast_dtype("cuda") == torch.bfloat16))

    def _w16_pair(self):
        """(bf16 W, bf16 Wᵀ): the model's LinearWeightPrep views when they are
        current, else the cached casts."""
        v = prepped_linear((self.weight,))
        if v is not None:
            return v
        w16 = self._bf16(self.weight, "_w16_cache")
        if w16 is None:
            w16 = self.weight.detach().to(torch.bfloat16)
        return w16, self._bf16t(w16)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._fast(x):
            w16, w16t = self._w16_pair()
            b16 = self._bf16(self.bias, "_b16_cache") if self.bias is not None else None
            return _LinearFn.apply(x, self.weight, self.bias, w16, b16, w16t)
        return super().forward(x)

    def forward_gelu(self, x: torch.Tensor, approximate: str = "none") -> torch.Tensor:
        """``F.gelu(self(x), approximate=approximate)`` with the GELU on our
        kernels and the bias gradient fused into the GELU backward."""
        if approximate not in ("none", "tanh"):
            raise ValueError(f"approximate must be 'none' or 'tanh', got {approximate!r}")
        if _FUSED_GELU and self._fast(x):
            w16, w16t = self._w16_pair()
            b16 = self._bf16(self.bias, "_b16_cache") if self.bias is not None else None
            return _LinearGeluFn.apply(x, self.weight, self.bias, w16, b16, w16t, approximate == "tanh")
        return F.gelu(self.forward(x), approximate=approximate)


def packed_linear(x: torch.Tensor, layers) -> torch.Tensor:
    """``torch.cat([l(x) for l in layers], -1)`` as ONE GEMM: one forward GEMM,
    one data-gradient GEMM whose K spans all the layers (no separate adds of
    the per-layer input gradients) and one weight-gradient GEMM; each layer
    keeps its own parameter, gradient and state_dict key. BERT's query / key /
    value projections: their packed output feeds the packed flash-attention
    entry point directly. With the model's :class:`LinearWeightPrep` current,
    the packed bf16 weight and its transpose come from its one launch per
    optimizer step (:class:`_PackedLinearFn`: no fp32 weight concatenation,
    cast or transpose per call); else the weights are concatenated here."""
    fast = x.is_cuda and all(l.in_features % 8 == 0 and l.out_features % 8 == 0 for l in layers) and (
        x.dtype == torch.bfloat16 or (torch.is_autocast_enabled("cuda")
                                      and torch.get_autocast_dtype("cuda") == torch.bfloat16))
    if fast and all(l.bias is not None for l in layers):
        v = prepped_linear(tuple(l.weight for l in layers))
        if v is not None:
            b = torch.cat([l.bias for l in layers], 0)
            return _PackedLinearFn.apply(x, b, v[0], v[1], *(l.weight for l in layers))
    w = torch.cat([l.weight for l in layers], 0)
    b = torch.cat([l.bias for l in layers], 0) if all(l.bias is not None for l in layers) else None
    if not fast or b is None:
        return F.linear(x, w, b)
    w16 = w.detach().to(torch.bfloat16)
    return _LinearFn.apply(x, w, b, w16, None, w16.t().contiguous())


class _PackedLinearFn(torch.autograd.Function):
    """y = x·[W₁; W₂; …]ᵀ + b over the row-packed bf16 weight (and its
    transpose) of a :class:`LinearWeightPrep` group; the packed fp32 weight
    gradient goes back to each member as its row slice."""

    @staticmethod
    def forward(ctx, x, bias, w16, w16t, *weights):
        x, w, b = _setup(ctx, x, weights[0], bias, w16, None)
        ctx.params = (None, bias)  # no in-place .grad add: the packed gradient is split by rows
        ctx.rows = [wt.shape[0] for wt in weights]
        ctx.weights = weights
        ctx.save_for_backward(x, w, w16t)
        return _linear_fwd(x, w, b, bias)

    @staticmethod
    def backward(ctx, gy):
        x, w, wt = ctx.saved_tensors
        gy = gy.contiguous()
        if gy.dtype != torch.bfloat16:
            gy = gy.to(torch.bfloat16)
        n = ctx.needs_input_grad
        sub = _Sub((n[0], any(n[4:]), n[1]), ctx.params, ctx.wdtype, ctx.bdtype, ctx.accum, ctx.defer,
                   ctx.weights, ctx.rows)
        dx, dw, db = _linear_backward(sub, gy.view(-1, gy.shape[-1]), x, w, wt=wt)
        dws = dw.split(ctx.rows, 0) if dw is not None else (None,) * len(ctx.rows)
        return (dx, db, None, None, *dws)


# weight -> (LinearWeightPrep, group index) for every weight a prep writes
_PREP_OF = WeakIdKeyDictionary()


def prepped_linear(weights: tuple):
    """(bf16 W, bf16 Wᵀ) of a weight — or of a row-packed group of weights —
    from the :class:`LinearWeightPrep` that owns it, when its buffer holds the
    weights' current values; else None."""
    e = _PREP_OF.get(weights[0])
    if e is None:
        return None
    return e[0].views(e[1], weights)


class LinearWeightPrep:
    """bf16 GEMM operands of a model's Linear weights, ALL written by ONE
    kernel launch per optimizer step (``weight_prep_kernel``, gemm.hip) into
    one persistent buffer: per weight — or per row-packed group (BERT's
    query / key / value) — the bf16 W [N, K] the forward GEMM reads and the
    bf16 Wᵀ [K, N] of the data gradient, through an LDS-tiled transpose. A
    group may be padded to ``pad_rows`` rows (zeros): the tied LM head's
    vocabulary is padded to a multiple of 64 so it runs on our GEMMs
    (:func:`lm_head_cross_entropy`).

    Replaces, per step, one cast launch per weight (or the fused optimizer's
    bf16 shadow write) plus one ATen strided-copy transpose per weight
    (0.59 ms of a GPT-2 step, profiles/r3_gpt2_copy_trace.log) and
    packed_linear's per-call fp32 concatenation, cast and transpose.

    :meth:`refresh` — called at the top of the model's forward — relaunches
    only when a weight changed (fused-optimizer epoch, autograd version) or
    while a HIP graph is being captured (the launch is then part of every
    replay; the buffer's addresses are fixed), and replans when a weight's
    storage moved. Readers (:func:`prepped_linear`) get the views only while
    they are current; otherwise they cast themselves. The backward keeps
    references to the buffer (saved tensors); the next rewrite happens after
    the optimizer step, i.e. after that backward.
    Reference parity: the ``nn.Linear`` layers of the BASELINE transformer
    configs."""

    def __init__(self, groups, pad_rows=None):
        self.groups = [tuple(g) for g in groups]
        self.pad_rows = [int(r) for r in pad_rows] if pad_rows is not None else [0] * len(self.groups)
        if len(self.pad_rows) != len(self.groups):
            raise ValueError("LinearWeightPrep: one pad_rows entry per group")
        for g in self.groups:
            for w in g:
                if not self.eligible(w):
                    raise ValueError("LinearWeightPrep: contiguous fp32 2-D CUDA weights with "
                                     f"multiples of 8 rows / columns required, got {tuple(w.shape)} {w.dtype}")
        self._ptrs = None
        self._epoch = None
        self._versions = None
        self._first = []  # group -> index of its first weight in the flat weight list
        k = 0
        for i, g in enumerate(self.groups):
            _PREP_OF[g[0]] = (self, i)
            self._first.append(k)
            k += len(g)

    @staticmethod
    def eligible(w: torch.Tensor) -> bool:
        return (w.is_cuda and w.dtype == torch.float32 and w.dim() == 2 and w.is_contiguous()
                and w.shape[1] % 8 == 0)

    @classmethod
    def for_model(cls, model: nn.Module, packed=(), heads=None) -> "LinearWeightPrep":
        """A prep over every eligible :class:`FusedLinear` of ``model`` (members
        of ``packed`` groups only as their group) plus ``heads`` ({weight:
        padded rows}: tied LM heads)."""
        packed = [tuple(g) for g in packed if all(cls.eligible(w) and w.shape[0] % 8 == 0 for w in g)
                  and len({w.shape[1] for w in g}) == 1]
        heads = {w: r for w, r in (heads or {}).items() if cls.eligible(w)}
        in_group = {id(w) for g in packed for w in g}
        groups, pads = [], []
        for m in model.modules():
            if isinstance(m, FusedLinear) and id(m.weight) not in in_group and cls.eligible(m.weight) \
                    and m.weight.shape[0] % 8 == 0:
                groups.append((m.weight,))
                pads.append(0)
        for g in packed:
            groups.append(g)
            pads.append(0)
        for w, rows in heads.items():
            groups.append((w,))
            pads.append(rows)
        return cls(groups, pads)

    @classmethod
    def attach(cls, model: nn.Module, packed=(), heads=None):
        """The model's prep, refreshed (a no-op while the weights are
        unchanged): built on the first call with the model on the GPU and
        rebuilt when a weight Parameter was replaced; None on the CPU."""
        p = model.__dict__.get("_linear_prep")
        if p is None or p._stale_params(model, packed, heads):
            if not any(m.weight.is_cuda for m in model.modules() if isinstance(m, FusedLinear)):
                return None
            p = cls.for_model(model, packed, heads)
            p._sig = cls._signature(model, packed, heads)
            model.__dict__["_linear_prep"] = p
        p.refresh()
        return p

    @staticmethod
    def _signature(model, packed, heads):
        return tuple(id(m.weight) for m in model.modules() if isinstance(m, FusedLinear)) + tuple(
            id(w) for g in packed for w in g) + tuple(id(w) for w in (heads or {}))

    def _stale_params(self, model, packed, heads) -> bool:
        return getattr(self, "_sig", None) != self._signature(model, packed, heads)

    def refresh(self) -> None:
        from ..optim.fused import param_epoch

        ws = [w for g in self.groups for w in g]
        ptrs = tuple(w.data_ptr() for w in ws)
        if ptrs != self._ptrs:
            self.table, self.tiles, self.wb, self.wt = _C.weight_prep_plan(
                [w.detach() for w in ws], [len(g) for g in self.groups], self.pad_rows)
            self._ptrs, self._epoch = ptrs, None
        capturing = torch.cuda.is_current_stream_capturing()
        versions = [w._version for w in ws]
        epoch = param_epoch()
        if capturing:
            # once per captured step: the micro-steps of a gradient-accumulation
            # step see the same weights (the optimizer, which changes them,
            # runs after the last one); a new capture or an optimizer step in
            # between launches again. Each replay re-preps from the weights
            # the previous replay's optimizer wrote.
            ckey = (_C.stream_capture_id(torch.cuda.current_stream().cuda_stream), epoch, tuple(versions))
            if ckey != getattr(self, "_cap_key", None):
                _C.weight_prep_run(self.table, self.tiles)
                self._cap_key = ckey
            self._epoch, self._versions = epoch, versions
        elif epoch != self._epoch or versions != self._versions:
            _C.weight_prep_run(self.table, self.tiles)
            self._epoch, self._versions = epoch, versions

    def views(self, i: int, weights: tuple):
        """(wb, wt) of group ``i`` if it is ``weights`` and current, else None."""
        from ..optim.fused import param_epoch

        g = self.groups[i]
        if self._epoch is None or len(g) != len(weights) or any(a is not b for a, b in zip(g, weights)):
            return None
        if param_epoch() != self._epoch or self._ptrs is None:
            return None
        k = self._first[i]
        for j, w in enumerate(g):
            if w._version != self._versions[k + j] or w.data_ptr() != self._ptrs[k + j]:
                return None
        return self.wb[i], self.wt[i]


class _Sub:
    """The per-Linear slice of an autograd ctx that _linear_backward reads."""

    def __init__(self, needs, params, wdtype, bdtype, accum, defer=False, defer_params=None, rows=None):
        self.needs_input_grad, self.params, self.wdtype, self.bdtype, self.accum = needs, params, wdtype, bdtype, accum
        self.defer, self.defer_params, self.rows = defer, defer_params, rows


class _MLPFn(torch.autograd.Function):
    """proj(gelu(fc(x))) as one node. Forward: fc with the bias + GELU
    epilogue (h and gelu(h) out of one GEMM), proj with the bias epilogue.
    Backward: proj's data gradient IS gelu(h)'s gradient, so its GEMM stores
    gh = (gy·W2)·gelu'(h) directly and sums fc's bias gradient in the same
    epilogue (``_C.linear_dgrad_gelu``, gemm.hip EPI 10/11): the separate
    GELU-backward pass over gy and h (50-100 MB per GPT-2 / BERT layer) is gone."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w1_16, b1_16, w2_16, w1t, w2t, tanh):
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        mode = 1 if tanh else 2
        x2 = x.reshape(-1, x.shape[-1])
        b1_32, b2_32 = _bias32(b1), _bias32(b2)
        c1 = _CHOICE.get(("fwd_gelu", x2.shape[0], w1_16.shape[1], w1_16.shape[0]), _DEFAULT_OURS)
        if c1 == "pp" and _pp_ok(x2.shape[0], w1_16.shape[0], w1_16.shape[1]):
            y1, h = _C.gemm_pp(x, w1_16, b1_32, mode)
        elif c1 == "hipblaslt":  # (the node's gain is its backward: any forward kernel will do)
            h = F.linear(x, w1_16, _lb(b1))
            y1 = _C.gelu_fwd(h, tanh)
        else:
            y1, h = _C.linear_fwd(x, w1_16, b1_32, mode)
        y1_2 = y1.reshape(-1, y1.shape[-1])
        c2 = _pick(("fwd", y1_2.shape[0], w2_16.shape[1], w2_16.shape[0]), _fwd_cands(y1_2, w2_16, b2, b2_32, 0))
        if c2 == "pp":
            out = _C.gemm_pp(y1, w2_16, b2_32, 0)[0]
        elif c2 == "ring":
            out = _C.linear_fwd(y1, w2_16, b2_32, 0)[0]
        else:
            out = F.linear(y1, w2_16, _lb(b2))
        ctx.save_for_backward(x, h, y1, w1_16, w2_16, w1t, w2t)
        ctx.tanh = tanh
        ctx.accum = accumulating()
        ctx.defer = deferring()
        _claim((w1, b1, w2, b2))
        ctx.wdtypes = (w1.dtype, w2.dtype)
        ctx.bdtypes = (b1.dtype, b2.dtype)
        ctx.params = (w1, b1, w2, b2)
        return out

    @staticmethod
    def backward(ctx, gout):
        x, h, y1, w1_16, w2_16, w1t, w2t = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        gout = gout.contiguous()
        if gout.dtype != torch.bfloat16:
            gout = gout.to(torch.bfloat16)
        g2 = gout.view(-1, gout.shape[-1])
        n = ctx.needs_input_grad
        # proj: weight / bias gradients as a plain Linear (no data gradient here)
        sub2 = _Sub((False, n[3], n[4]), (w2, b2), ctx.wdtypes[1], ctx.bdtypes[1], ctx.accum, ctx.defer)
        _, dw2, db2 = _linear_backward(sub2, g2, y1, w2_16)
        # proj's data gradient with the GELU backward and fc's bias sum fused in
        tgt = _acc_target(ctx, b1, torch.Size((h.shape[-1],))) if n[2] else None
        M, N1, N2 = g2.shape[0], h.shape[-1], g2.shape[1]
        pp = _CHOICE.get(("mlp_bwd", M, N2, N1)) == "pp" and _pp_ok(M, N1, N2) and N1 % 8 == 0
        gh, db1 = _C.linear_dgrad_gelu(g2, w2t, h.view(-1, h.shape[-1]), ctx.tanh, accumulate_into=tgt, pp=pp)
        if tgt is not None or not n[2]:
            db1 = None
        elif db1.dtype != ctx.bdtypes[0]:
            db1 = db1.to(ctx.bdtypes[0])
        sub1 = _Sub((n[0], n[1], n[2]), (w1, b1), ctx.wdtypes[0], ctx.bdtypes[0], ctx.accum, ctx.defer)
        dx, dw1, _ = _linear_backward(sub1, gh, x, w1_16, db=db1, db_done=True, wt=w1t)
        return dx, dw1, db1, dw2, db2, None, None, None, None, None, None


def _mlp_prefers_ours(x, w1_16, b1, b1_16, w2_16, w2t, tanh) -> bool:
    """Whether the MLP runs as the fused node (:class:`_MLPFn`). The node's
    gain is in its backward: proj's data gradient with the GELU backward and
    fc's bias-gradient sums in the ring GEMM's epilogue (``linear_dgrad_gelu``)
    instead of the fastest plain data-gradient GEMM (pp / ring / hipBLASLt)
    plus the separate GELU-backward pass over gy and h. Both are timed
    (``("mlp_bwd", M, N2, N1)``: "ring" / "pp" = fused on the ring / the
    ping-pong GEMM's GELU-backward epilogue, "hipblaslt" = unfused — the names
    the autotune table already carries); its forward takes whichever
    kernel the fc forward autotune picked."""
    M, K = x.numel() // x.shape[-1], x.shape[-1]
    N1, N2 = w1_16.shape[0], w2_16.shape[0]
    key_f, key_d, key_b = ("fwd_gelu", M, K, N1), ("dgrad", M, N2, N1), ("mlp_bwd", M, N2, N1)
    if key_b not in _CHOICE:
        if not _AUTOTUNE or torch.cuda.is_current_stream_capturing():
            return True
        mode = 1 if tanh else 2
        with torch.no_grad():
            x2 = x.detach().reshape(M, K).to(torch.bfloat16)
            if key_f not in _CHOICE:
                _pick(key_f, _fwd_cands(x2, w1_16, b1_16, _bias32(b1), mode))
            # private generator: the stand-in gradient / pre-activation must not
            # move the global RNG stream that dropout / init draw from
            gen = torch.Generator(device=x.device).manual_seed(0)
            g2 = torch.empty(M, N2, device=x.device, dtype=torch.bfloat16).normal_(generator=gen)
            h = torch.empty(M, N1, device=x.device, dtype=torch.bfloat16).normal_(generator=gen)
            dc = _dgrad_cands(g2, w2_16, w2t)
            best = _pick(key_d, dc)

            def unfused():
                gy = dc[best]()
                return _C.gelu_bwd(gy[0] if isinstance(gy, (list, tuple)) else gy, h, tanh, True)

            cands = {"ring": lambda: _C.linear_dgrad_gelu(g2, w2t, h, tanh), "hipblaslt": unfused}
            if _pp_ok(M, N1, N2) and N1 % 8 == 0:
                cands["pp"] = lambda: _C.linear_dgrad_gelu(g2, w2t, h, tanh, pp=True)
            _pick(key_b, cands)
    return _CHOICE[key_b] != "hipblaslt"


def fused_mlp_gelu(x: torch.Tensor, fc: "FusedLinear", proj: "FusedLinear", approximate: str = "none"):
    """``proj(F.gelu(fc(x), approximate))`` — one autograd node (:class:`_MLPFn`)
    on the fast path (bf16 GPU, GEMM-able shapes), else the two modules."""
    if approximate not in ("none", "tanh"):
        raise ValueError(f"approximate must be 'none' or 'tanh', got {approximate!r}")
    ok = (_FUSED_MLP and _FUSED_GELU and _OUR_FWD and _OUR_DGRAD and isinstance(fc, FusedLinear) and isinstance(proj, FusedLinear)
          and fc._fast(x) and x.is_contiguous() and x.numel() > 0 and fc.bias is not None and proj.bias is not None
          and fc.out_features % 64 == 0 and fc.in_features % 64 == 0 and proj.out_features % 64 == 0
          and fc.in_features <= 4096 and proj.in_features <= 4096 and proj.out_features <= 4096
          and proj.in_features == fc.out_features)
    if ok:
        w1_16, w1t = fc._w16_pair()
        w2_16, w2t = proj._w16_pair()
        b1_16 = fc._bf16(fc.bias, "_b16_cache")
        # the fused node's backward (dgrad + GELU backward in one ring GEMM)
        # against the fastest plain dgrad + the separate GELU pass, timed
        ok = _mlp_prefers_ours(x, w1_16, fc.bias, b1_16, w2_16, w2t, approximate == "tanh")
    if not ok:
        return proj(fc.forward_gelu(x, approximate) if isinstance(fc, FusedLinear) else
                    F.gelu(fc(x), approximate=approximate))
    return _MLPFn.apply(x, fc.weight, fc.bias, proj.weight, proj.bias, w1_16, b1_16, w2_16, w1t, w2t,
                        approximate == "tanh")
