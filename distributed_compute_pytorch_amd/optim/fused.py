"""Fused multi-tensor optimizers (one HIP launch per parameter group class).

Parity: ``optim.Adadelta(model.parameters(), lr=opt.lr)`` at main.py:124
(SURVEY §2b F14, §2f K25 — ~100 kernel launches per step in the reference),
plus SGD (ResNet-50 config) and Adam/AdamW (BERT / GPT-2 configs). These are
``torch.optim.Optimizer`` subclasses, so ``state_dict()`` / ``load_state_dict``
/ ``zero_grad`` / LR schedulers (``StepLR``, main.py:125) behave exactly like
torch's, and the per-parameter state keys match torch
(``momentum_buffer``; ``step``/``exp_avg``/``exp_avg_sq``[/``max_exp_avg_sq``];
``step``/``square_avg``/``acc_delta``).

The update math runs in fp32 registers for fp32/bf16/fp16 parameters; state
dtype follows the parameter (as in torch).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Iterable, List, Optional

import os

import torch
from torch.optim import Optimizer
from torch.utils.weak import WeakIdKeyDictionary

from .._ext import C as _C


# Bumped by every fused step: the kernels update parameters through raw
# pointers (no autograd version bump), so caches of derived tensors (the bf16
# weight copies of ops.linear.FusedLinear) key on this as well as _version.
_PARAM_EPOCH = [0]


def param_epoch() -> int:
    return _PARAM_EPOCH[0]


# fp32 parameter -> [bf16 shadow, epoch, _version]: bf16 copies that the
# consumer (ops.linear.FusedLinear) registers once; the fused Adam/AdamW kernel
# then rewrites them with the updated weights in the same pass as the update
# (no separate cast launch per weight per step — 150 launches / 0.7 ms of a
# BERT-base step, profiles/r1_bert_prof71_gelu.txt). A shadow is valid only
# while (epoch, _version) match, i.e. nobody modified the parameter since.
_BF16_SHADOWS = WeakIdKeyDictionary()


def register_bf16_shadow(p: torch.Tensor, shadow: torch.Tensor) -> None:
    if p.dtype == torch.float32 and p.is_cuda and p.is_contiguous() and shadow.shape == p.shape:
        _BF16_SHADOWS[p] = [shadow, _PARAM_EPOCH[0], p._version]


def fresh_bf16_shadow(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The registered shadow of ``p`` if it holds p's current values."""
    e = _BF16_SHADOWS.get(p)
    if e is not None and e[1] == _PARAM_EPOCH[0] and e[2] == p._version:
        return e[0]
    return None


def _overlap_chunks(opt, ranges_ok: bool = False):
    """Optimizer overlap (``DistributedDataParallel(overlap_optimizer=True)``):
    when a DDP left bucket reductions deferred, the step runs in chunks —
    first every parameter outside those buckets, then bucket by bucket in
    launch order, each right after the compute stream is ordered behind that
    bucket's collective (``sync``) — so the updates of the early buckets run
    while the last ones are still being reduced. None when nothing is deferred.

    Chunks are ``(sync, ids, ranges)``. With ``ranges_ok`` (an optimizer that
    can update part of a parameter: Adam / AdamW) a bucket the Reducer
    reduced slice by slice (``bucket_slice_mb``: GPT-2's 147 MB tied
    embedding) gives one chunk per slice: the parameters wholly inside the
    slice in ``ids``, and ``ranges`` = {id(p): (lo, hi)} — the flat element
    range of each parameter the slice only partly covers, in slice order."""
    from ..parallel import ddp as _ddp

    chunks, covered = [], set()
    for d in list(_ddp._OVERLAP):
        plan = None
        for k in d.reducer.deferred_buckets():
            if plan is None:
                plan = d.reducer.bucket_indices()
            ps = [d._params[i] for i in plan[k]]
            ids = {id(p) for p in ps}
            covered |= ids
            bounds = d.reducer.bucket_slice_bounds(k) if ranges_ok else []
            if not bounds:
                chunks.append((lambda d=d, k=k: d.reducer.sync_bucket(k), ids, None))
                continue
            ns = len(bounds) - 1
            whole = [set() for _ in range(ns)]
            part = [{} for _ in range(ns)]
            o, s = 0, 0
            for p in ps:  # the bucket's flat layout: parameters back to back
                n = p.numel()
                while s < ns - 1 and bounds[s + 1] <= o:
                    s += 1
                t = s
                while t < ns - 1 and bounds[t + 1] < o + n:
                    t += 1
                if t == s:
                    whole[s].add(id(p))
                else:
                    for u in range(s, t + 1):
                        part[u][id(p)] = (max(o, bounds[u]) - o, min(o + n, bounds[u + 1]) - o)
                o += n
            for u in range(ns):
                chunks.append((lambda d=d, k=k, u=u: d.reducer.sync_bucket_slice(k, u), whole[u], part[u]))
    if not chunks:
        return None
    mine = {id(g_p) for g in opt.param_groups for g_p in g["params"]}
    out = [(None, mine - covered, None)]
    for sync, ids, ranges in chunks:
        out.append((sync, ids & mine, {i: r for i, r in ranges.items() if i in mine} if ranges else None))
    return out


def _run_chunks(opt, impl, grad_scale, ranged=None) -> list:
    """``impl(ids, grad_scale)`` over the overlap chunks (one call with ids =
    None when nothing is deferred), and ``ranged(ranges, grad_scale)`` for
    the partial-parameter ranges of sliced buckets (optimizers that pass
    one); the list of the results."""
    out = []
    for sync, ids, ranges in _overlap_chunks(opt, ranged is not None) or [(None, None, None)]:
        if sync is not None:
            sync()
        if ids is None or ids:
            out.append(impl(ids, grad_scale))
        if ranges:
            out.append(ranged(ranges, grad_scale))
    return out


def sync_deferred_gradients() -> None:
    """Order the current stream behind every deferred bucket reduction of every
    overlap-mode DDP (anything that reads .grad outside the fused optimizers'
    step — e.g. gradient clipping — must call this first)."""
    from ..parallel import ddp as _ddp

    for d in list(_ddp._OVERLAP):
        d.wait_gradients()


def _chunk_params(opt, group, ids):
    """The group's parameters in ``ids`` (all when None), without scanning the
    whole group per overlap chunk: a per-group id -> parameter map, rebuilt
    when the group's parameter list changes."""
    if ids is None:
        return group["params"]
    cache = opt.__dict__.setdefault("_dcp_idmaps", {})
    params = group["params"]
    key = id(group)
    hit = cache.get(key)
    if hit is None or hit[0] is not params or hit[1] != len(params):
        hit = cache[key] = (params, len(params), {id(p): (i, p) for i, p in enumerate(params)})
    found = [hit[2][i] for i in ids if i in hit[2]]
    found.sort(key=lambda t: t[0])  # group order (what a full scan would visit)
    return [p for _, p in found]


def _grad(p: torch.Tensor):
    """p.grad — for an overlap-mode DDP's pending gradient (parallel/ddp.py
    _PendingGrad) the plain bucket view behind it, without the sync a torch op
    on the wrapper performs: the step's chunk for that bucket has just synced
    it (_run_chunks), and only the bucket's own sync may be waited for."""
    g = p.grad
    if g is not None and type(g).__name__ == "_PendingGrad":
        return g.__dict__["_dcp_plain"]
    return g


def _grads_ok(p: torch.Tensor) -> bool:
    g = _grad(p)
    if g is None:
        return False
    if g.is_sparse:
        raise RuntimeError("fused optimizers do not support sparse gradients")
    return True


def _dense_like(g: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """The kernels stream memory in order: grad layout must equal the param's."""
    if g.stride() == p.stride() or (g.is_contiguous() and p.is_contiguous()):
        return g
    return torch.empty_like(p, memory_format=torch.preserve_format).copy_(g)


def _state_like(p: torch.Tensor) -> torch.Tensor:
    return torch.zeros_like(p, memory_format=torch.preserve_format)


class _DropsDeferred:
    """zero_grad also drops the micro-step weight-gradient contributions a
    ``defer_accum_wgrad`` DDP still holds for these parameters (they are part
    of ``.grad``, only not yet added into it: ops/linear.py)."""

    def zero_grad(self, set_to_none: bool = True):
        from ..ops import linear as _lin

        if _lin.pending_weight_grads():
            _lin.discard_weight_grads([p for g in self.param_groups for p in g["params"]])
        super().zero_grad(set_to_none)


class SGD(_DropsDeferred, Optimizer):
    """torch.optim.SGD semantics, fused multi-tensor update."""

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, *, maximize: bool = False):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        _run_chunks(self, self._step, grad_scale)
        _PARAM_EPOCH[0] += 1
        return loss

    def _step(self, ids, grad_scale):
        """Update the parameters whose id is in ``ids`` (None: all)."""
        for group in self.param_groups:
            mom = group["momentum"]
            buckets = defaultdict(lambda: ([], [], []))
            capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
            for p in group["params"]:
                if (ids is not None and id(p) not in ids) or not _grads_ok(p):
                    continue
                st = self.state[p]
                first = False
                if mom != 0 and st.get("momentum_buffer") is None:
                    if capturing:
                        # a captured "first step" flag would re-initialise the
                        # buffer on every replay: start from zeros instead
                        # (identical update when dampening == 0)
                        if group["dampening"] != 0:
                            raise RuntimeError("SGD with dampening cannot take its first step inside HIP-graph "
                                               "capture: run one eager step (warmup) before capturing")
                        st["momentum_buffer"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    else:
                        st["momentum_buffer"] = torch.empty_like(p, memory_format=torch.preserve_format)
                        first = True
                key = (p.device, p.dtype, first)
                P, G, B = buckets[key]
                P.append(p)
                G.append(_dense_like(_grad(p), p))
                if mom != 0:
                    B.append(st["momentum_buffer"])
            for (dev, dt, first), (P, G, B) in buckets.items():
                _C.fused_sgd(P, G, B, group["lr"], mom, group["dampening"], group["weight_decay"],
                             group["nesterov"], group["maximize"], first, grad_scale)


class Adam(_DropsDeferred, Optimizer):
    """torch.optim.Adam / AdamW semantics (``decoupled_weight_decay``), fused.

    ``capturable=True`` (torch's flag of the same name): every parameter's
    ``step`` lives on the device, is advanced by one launch per step and the
    kernel derives the bias corrections from it, so a step captured in a HIP
    graph keeps advancing on replay. Without it the bias corrections are host
    constants, and stepping inside a capture raises instead of silently
    freezing them. A group can be switched at any time; the state migrates on
    its next eager step.
    """

    _decoupled_default = False

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, *, maximize: bool = False, decoupled_weight_decay: bool = None,
                 capturable: bool = False):
        if decoupled_weight_decay is None:
            decoupled_weight_decay = self._decoupled_default
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        decoupled_weight_decay=decoupled_weight_decay, capturable=capturable)
        super().__init__(params, defaults)

    def __setstate__(self, state):
        super().__setstate__(state)
        for g in self.param_groups:
            g.setdefault("capturable", False)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        shadowed = [p for sh in _run_chunks(self, self._step, grad_scale, self._step_ranges) for p in sh]
        _PARAM_EPOCH[0] += 1
        for p in shadowed:  # rewritten by the kernel: valid for the new epoch
            e = _BF16_SHADOWS[p]
            e[1], e[2] = _PARAM_EPOCH[0], p._version
        return loss

    def _step(self, ids, grad_scale):
        """Update the parameters whose id is in ``ids`` (None: all); returns the
        parameters whose bf16 shadow the kernel rewrote.

        Host cost: the per-parameter work (state lookup and migration, bucket
        grouping, argument lists) is done once per chunk and cached as a plan,
        revalidated each step from the gradients' addresses / layouts and the
        bf16 shadows (`_adam_sig`); the host-side step counters of a plan are
        0-dim views of one flat CPU tensor, advanced by a single add. Before,
        the per-parameter loop and counter updates were ~1.5 ms of host time
        per BERT step, spent while the GPU idled between the backward's last
        kernel and the first update (NOTES §28)."""
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        shadowed = []
        plans = self.__dict__.setdefault("_dcp_plans", {})
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            ams = group["amsgrad"]
            cap_mode = group.get("capturable", False)
            if capturing and not cap_mode:
                raise RuntimeError("Adam/AdamW stepped inside HIP-graph capture without capturable=True: the "
                                   "bias corrections would be frozen at their capture-time step. Construct the "
                                   "optimizer with capturable=True (or set group['capturable'] = True before the "
                                   "eager warmup steps).")
            plist = _chunk_params(self, group, ids)
            grads, sig = _adam_sig(plist)
            pkey = (gi, id(group), None if ids is None else tuple(id(p) for p in plist), cap_mode, ams)
            plan = plans.get(pkey)
            if (plan is None or plan.sig != sig or plan.state is not self.state or capturing or _NO_PLAN
                    or not plan.counters_live()):
                plan = self._adam_plan(plist, grads, cap_mode, ams, capturing)
                plan.sig = sig
                if plan.cacheable and not capturing:
                    plans[pkey] = plan
                else:
                    plans.pop(pkey, None)
            vals = None
            if plan.flat is not None:
                plan.flat.add_(1.0)  # every host-side step counter of the plan, one op
                vals = plan.flat.tolist()
            for bk in plan.buckets:
                if bk.st:
                    torch._foreach_add_(bk.st, 1.0)  # one launch; the kernel reads the advanced steps
                    step = 0.0
                else:
                    step = vals[bk.steps[0]]
                    if any(vals[i] != step for i in bk.steps):  # a counter edited by hand: regroup next step
                        plans.pop(pkey, None)
                        for i in bk.steps:
                            self._adam_one(plist, grads, i, vals[i], group, b1, b2, ams, grad_scale)
                        shadowed.extend(bk.shadowed)
                        continue
                g = [grads[i] for i in bk.idx]
                _C.fused_adam(bk.p, g, bk.m, bk.v, bk.vm, group["lr"], b1, b2, group["eps"], group["weight_decay"],
                              step, ams, group["decoupled_weight_decay"], group["maximize"], grad_scale, bk.s, bk.st)
                shadowed.extend(bk.shadowed)
        return shadowed

    def _step_ranges(self, ranges, grad_scale):
        """Update flat element ranges of parameters (``ranges`` = {id(p): (lo,
        hi)}, overlap chunks of a bucket reduced slice by slice): Adam is
        elementwise, so a range update with the parameter's step equals the
        whole-tensor update on those elements. The step counter advances at
        the range starting at 0 (ranges come in slice order). A parameter that
        cannot be updated in ranges (no state yet, capturable, non-contiguous)
        is updated whole at its last range, when all its slices have landed.
        Returns the parameters whose bf16 shadow the kernel rewrote."""
        shadowed = []
        where = {}
        for group in self.param_groups:
            for p in group["params"]:
                if id(p) in ranges:
                    where[id(p)] = (group, p)
        for pid, (lo, hi) in ranges.items():
            if pid not in where:
                continue
            group, p = where[pid]
            g = _grad(p)
            if g is None:
                continue
            st = self.state[p]
            last = hi == p.numel()
            ams = group["amsgrad"]
            ok = (len(st) > 0 and not group.get("capturable", False) and not st["step"].is_cuda
                  and p.is_contiguous() and g.is_contiguous() and not g.is_sparse
                  and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()
                  and (not ams or st["max_exp_avg_sq"].is_contiguous()))
            sh = _BF16_SHADOWS.get(p) if p.is_cuda else None
            if ok and sh is not None and not sh[0].is_contiguous():
                ok = False
            if not ok:
                if last:
                    shadowed.extend(self._step({pid}, grad_scale))
                continue
            if lo == 0:
                st["step"].add_(1.0)  # in place: the value a cached plan's flat counters share
            b1, b2 = group["betas"]

            def r(t):
                return t.view(-1)[lo:hi]

            _C.fused_adam([r(p)], [r(g)], [r(st["exp_avg"])], [r(st["exp_avg_sq"])],
                          [r(st["max_exp_avg_sq"])] if ams else [], group["lr"], b1, b2, group["eps"],
                          group["weight_decay"], float(st["step"]), ams, group["decoupled_weight_decay"],
                          group["maximize"], grad_scale, [r(sh[0])] if sh is not None else [], [])
            if sh is not None and last:
                shadowed.append(p)
        return shadowed

    def _adam_one(self, plist, grads, i, step, group, b1, b2, ams, grad_scale):
        p = plist[i]
        st = self.state[p]
        sh = _BF16_SHADOWS.get(p) if p.is_cuda else None
        _C.fused_adam([p], [grads[i]], [st["exp_avg"]], [st["exp_avg_sq"]],
                      [st["max_exp_avg_sq"]] if ams else [], group["lr"], b1, b2, group["eps"], group["weight_decay"],
                      step, ams, group["decoupled_weight_decay"], group["maximize"], grad_scale,
                      [sh[0]] if sh is not None else [], [])

    def _adam_plan(self, plist, grads, cap_mode, ams, capturing):
        """State creation / migration and the launch grouping of one chunk."""
        plan = _AdamPlan()
        plan.state = self.state
        entries, cpu = [], []
        for i, p in enumerate(plist):
            if grads[i] is None:
                continue
            st = self.state[p]
            dev_step = cap_mode and p.is_cuda
            if len(st) == 0:
                st["step"] = (torch.zeros((), dtype=torch.float32, device=p.device) if dev_step
                              else torch.tensor(0.0, dtype=torch.float32))
                st["exp_avg"] = _state_like(p)
                st["exp_avg_sq"] = _state_like(p)
                if ams:
                    st["max_exp_avg_sq"] = _state_like(p)
            elif dev_step and not st["step"].is_cuda:
                if capturing:
                    raise RuntimeError("capturable Adam: run one eager step before capture (moves 'step' "
                                       "to the device)")
                st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
            elif not dev_step and st["step"].is_cuda:
                st["step"] = st["step"].cpu()
            dense = _dense_like(grads[i], p)
            if dense is not grads[i]:  # a layout copy: valid for this step only
                grads[i] = dense
                plan.cacheable = False
            entries.append((i, p, st, dev_step))
            if not dev_step:
                cpu.append(st)
        if cpu:
            # the counters as 0-dim views of one flat tensor (values kept; a
            # checkpoint still holds one 'step' tensor per parameter)
            plan.flat = torch.tensor([float(st["step"]) for st in cpu], dtype=torch.float32)
            for j, st in enumerate(cpu):
                st["step"] = plan.flat[j]
            plan.cpu = [(st, st["step"]) for st in cpu]
        vals = plan.flat.tolist() if cpu else []
        buckets = {}
        j = 0
        for i, p, st, dev_step in entries:
            sh = _BF16_SHADOWS.get(p) if p.is_cuda else None
            if dev_step:
                key = (p.device, p.dtype, None, sh is not None)
            else:
                key = (p.device, p.dtype, vals[j], sh is not None)
            bk = buckets.get(key)
            if bk is None:
                bk = buckets[key] = _AdamBucket()
            bk.idx.append(i)
            bk.p.append(p)
            bk.m.append(st["exp_avg"])
            bk.v.append(st["exp_avg_sq"])
            if ams:
                bk.vm.append(st["max_exp_avg_sq"])
            if sh is not None:
                bk.s.append(sh[0])
                bk.shadowed.append(p)
            if dev_step:
                bk.st.append(st["step"].view(1))
            else:
                bk.steps.append(j)
                j += 1
        plan.buckets = list(buckets.values())
        return plan


_NO_PLAN = os.environ.get("DCP_ADAM_NO_PLAN") == "1"  # A/B switch: rebuild the plan every step


class _AdamBucket:
    __slots__ = ("idx", "p", "m", "v", "vm", "s", "st", "steps", "shadowed")

    def __init__(self):
        self.idx, self.p, self.m, self.v, self.vm, self.s, self.st, self.steps, self.shadowed = (
            [], [], [], [], [], [], [], [], [])


class _AdamPlan:
    __slots__ = ("sig", "state", "flat", "buckets", "cacheable", "cpu")

    def __init__(self):
        self.sig, self.state, self.flat, self.buckets, self.cacheable, self.cpu = None, None, None, [], True, []

    def counters_live(self) -> bool:
        """True while every host-side 'step' of the plan is still its own view
        of ``flat``. Plans over overlapping parameter sets (the whole group and
        the overlap chunks of ``DistributedDataParallel(overlap_optimizer=True)``)
        each re-point the counters to their own flat tensor when built; a plan
        whose counters another plan took over is stale and must be rebuilt
        (from the current values), or it would advance its own copy."""
        return all(st.get("step") is v for st, v in self.cpu)


def _adam_sig(plist):
    """(grads, signature): each parameter's gradient (the plain bucket view for
    an overlap-mode pending gradient) and what a cached plan depends on — the
    gradient's address and layout and the bf16 shadow it updates."""
    grads, sig = [], []
    for p in plist:
        g = p.grad
        if g is None:
            grads.append(None)
            sig.append(None)
            continue
        if type(g).__name__ == "_PendingGrad":
            g = g.__dict__["_dcp_plain"]
        if g.is_sparse:
            raise RuntimeError("fused optimizers do not support sparse gradients")
        sh = _BF16_SHADOWS.get(p)
        grads.append(g)
        sig.append((g.data_ptr(), g.stride(), id(sh[0]) if sh is not None else 0))
    return grads, tuple(sig)


class AdamW(Adam):
    _decoupled_default = True

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 amsgrad: bool = False, *, maximize: bool = False, capturable: bool = False):
        super().__init__(params, lr, betas, eps, weight_decay, amsgrad, maximize=maximize, decoupled_weight_decay=True,
                         capturable=capturable)


class Adadelta(_DropsDeferred, Optimizer):
    """torch.optim.Adadelta semantics (reference optimizer, main.py:124), fused."""

    def __init__(self, params, lr: float = 1.0, rho: float = 0.9, eps: float = 1e-6, weight_decay: float = 0.0,
                 *, maximize: bool = False):
        defaults = dict(lr=lr, rho=rho, eps=eps, weight_decay=weight_decay, maximize=maximize)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        _run_chunks(self, self._step, grad_scale)
        _PARAM_EPOCH[0] += 1
        return loss

    def _step(self, ids, grad_scale):
        for group in self.param_groups:
            buckets = defaultdict(lambda: ([], [], [], []))
            for p in group["params"]:
                if (ids is not None and id(p) not in ids) or not _grads_ok(p):
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["square_avg"] = _state_like(p)
                    st["acc_delta"] = _state_like(p)
                st["step"] += 1
                P, G, S, A = buckets[(p.device, p.dtype)]
                P.append(p)
                G.append(_dense_like(_grad(p), p))
                S.append(st["square_avg"])
                A.append(st["acc_delta"])
            for _, (P, G, S, A) in buckets.items():
                _C.fused_adadelta(P, G, S, A, group["lr"], group["rho"], group["eps"], group["weight_decay"],
                                  group["maximize"], grad_scale)


@torch.no_grad()
def clip_grad_norm_(parameters: Iterable[torch.Tensor], max_norm: float, eps: float = 1e-6) -> torch.Tensor:
    """Total-L2-norm gradient clipping without a host sync: one sum-of-squares
    launch + one scale launch (the scale factor stays on device)."""
    sync_deferred_gradients()
    grads: List[torch.Tensor] = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    ss = _C.sumsq(grads)
    norm = ss[0].sqrt()
    coef = torch.clamp(max_norm / (norm + eps), max=1.0).reshape(1).to(torch.float32)
    _C.scale_by(grads, coef)
    return norm
