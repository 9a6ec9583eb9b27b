"""ZeRO-3 gathered-parameter residency plan (which all-gathered units stay in HBM between visits).

DeepSpeed decides this at run time from a parameter-fetch trace, driven by three
keys the reference's config generator emits (``ai_engine/deepspeed_launcher.py:188-190``):

* ``stage3_max_reuse_distance`` -- keep a gathered parameter if it is needed again
  within this many fetched parameters;
* ``stage3_max_live_parameters`` -- cap on the gathered parameters kept resident;
* ``stage3_prefetch_bucket_size`` -- how far ahead gathers are issued.

Our engine visits units in a fixed order (forward 0..n-1, backward n-1..0, repeated
per micro-batch), so the plan is computed once, exactly, at engine build time. With
288 GB of HBM per MI355X the ``"hbm"`` setting sizes the live budget to a fraction of
the device: a whole Llama-3-8B (16 GB bf16) then stays gathered across all
micro-batches of an optimizer step, i.e. ONE all-gather per unit per step instead
of two per micro-batch, while every piece of persistent state (bf16 parameters,
fp32 master / exp_avg / exp_avg_sq, fp32 gradients) stays partitioned 1/W.
"""
from __future__ import annotations

import math
from typing import Any, Callable, Dict, List, Sequence, Tuple


def resolve_limit(value: Any, hbm_params: Callable[[], float], unbounded_for_hbm: bool = False) -> float:
    """A knob value in parameters: a number, or "hbm" (sized from the device by `hbm_params`)."""
    if isinstance(value, str):
        if value not in ("hbm", "auto"):
            raise ValueError(f"ZeRO-3 residency knob must be a number or 'hbm', got {value!r}")
        return math.inf if unbounded_for_hbm else hbm_params()
    return float(value)


class ResidencyPlan:
    """keep(v, gi): does group gi stay gathered after visit v of a micro-step?

    ``visits[v]`` is the tuple of group indices visited at step v of one micro-batch
    (forward stages, then backward stages in reverse). ``sizes[gi]`` is the element count
    of group gi and ``gathered[gi]`` whether it is all-gathered at all (P > 1).

    The reuse distance of (v, gi) is the number of gathered parameters fetched before gi's
    next visit, wrapping into the next micro-batch. Candidates are admitted shortest distance
    first while the resident set stays within ``max_live``; a group counts once however many
    of its visits are kept.
    """

    def __init__(self, visits: Sequence[Tuple[int, ...]], sizes: Sequence[int], gathered: Sequence[bool],
                 max_live: float, max_reuse: float):
        self.visits = [tuple(v) for v in visits]
        self.max_live, self.max_reuse = max_live, max_reuse
        L = len(self.visits)
        fetched = [sum(sizes[g] for g in gis if gathered[g]) for gis in self.visits]
        self.distance: Dict[Tuple[int, int], int] = {}
        self.wraps: Dict[Tuple[int, int], bool] = {}
        cands: List[Tuple[int, int, int]] = []
        for v, gis in enumerate(self.visits):
            for gi in gis:
                if not gathered[gi]:
                    continue
                d, k = 0, 1
                while k < L and gi not in self.visits[(v + k) % L]:
                    d += fetched[(v + k) % L]
                    k += 1
                self.distance[(v, gi)] = d
                self.wraps[(v, gi)] = v + k >= L
                if d <= max_reuse:
                    cands.append((d, v, gi))
        self._keep: Dict[Tuple[int, int], bool] = {}
        resident, used = set(), 0
        for _, v, gi in sorted(cands):
            if gi in resident or used + sizes[gi] <= max_live:
                if gi not in resident:
                    resident.add(gi)
                    used += sizes[gi]
                self._keep[(v, gi)] = True
        self.resident_groups = sorted(resident)
        self.resident_params = used

    def held_through_step(self, gi: int) -> bool:
        """Every visit of gathered group gi is kept: one all-gather per step, the copy stays put until the
        optimizer step (what lets ZeRO-3 give it a transposed-weight cache, ZeroEngine._add_resident_tcache)."""
        vs = [v for v, gis in enumerate(self.visits) if gi in gis]
        return bool(vs) and all(self._keep.get((v, gi), False) for v in vs)

    def keep(self, v: int, gi: int, last_micro: bool) -> bool:
        """After the last micro-batch nothing survives a wrap: the optimizer step changes the parameters."""
        if not self._keep.get((v, gi), False):
            return False
        return not (last_micro and self.wraps[(v, gi)])

    def gathers_per_step(self, grad_accum: int) -> int:
        """All-gathers one optimizer step issues under this plan (for reports and tests)."""
        L = len(self.visits)
        live: set = set()
        n = 0
        for m in range(grad_accum):
            last = m == grad_accum - 1
            for v in range(L):
                for gi in self.visits[v]:
                    if (v, gi) not in self.wraps:
                        continue  # not gathered
                    if gi not in live:
                        n += 1
                        live.add(gi)
                for gi in self.visits[v]:
                    if (v, gi) in self.wraps and not self.keep(v, gi, last):
                        live.discard(gi)
        return n
