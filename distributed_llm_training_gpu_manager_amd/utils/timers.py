"""Per-phase wall-clock breakdown (the reference config's ``wall_clock_breakdown``,
``ai_engine/deepspeed_launcher.py`` emits it at ``generate_config``).

GPU phases are bracketed with HIP events recorded on the current stream, so timing
adds no host synchronisation to the step: elapsed times are resolved lazily in
:meth:`PhaseTimers.summary`, which the trainer calls at its log interval.
"""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Dict, List, Tuple

import torch


class PhaseTimers:
    def __init__(self, device: torch.device, enabled: bool = True):
        self.enabled = enabled
        self.cuda = device.type == "cuda"
        self._pending: List[Tuple[str, object, object]] = []
        self._acc: Dict[str, float] = defaultdict(float)
        self._cnt: Dict[str, int] = defaultdict(int)

    @contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        if self.cuda:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            try:
                yield
            finally:
                b.record()
                self._pending.append((name, a, b))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._pending.append((name, t0, time.perf_counter()))

    def mark(self):
        """A timestamp on the current stream (HIP event) -- pair two with :meth:`span`."""
        if not self.enabled:
            return None
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def span(self, name: str, a, b) -> None:
        if self.enabled and a is not None and b is not None:
            self._pending.append((name, a, b))

    def _resolve(self) -> None:
        for name, a, b in self._pending:
            if self.cuda:
                b.synchronize()
                ms = a.elapsed_time(b)
            else:
                ms = (b - a) * 1e3
            self._acc[name] += ms
            self._cnt[name] += 1
        self._pending.clear()

    def summary(self, reset: bool = True) -> Dict[str, Dict[str, float]]:
        """{phase: {"total_ms", "count", "mean_ms"}} since the last reset."""
        self._resolve()
        out = {k: {"total_ms": round(v, 3), "count": self._cnt[k], "mean_ms": round(v / max(1, self._cnt[k]), 3)}
               for k, v in self._acc.items()}
        if reset:
            self._acc.clear()
            self._cnt.clear()
        return out
