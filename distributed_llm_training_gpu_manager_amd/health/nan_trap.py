"""On-device NaN/Inf gradient trap (BASELINE config 3).

The engine's ``grad_stats`` kernel writes ``[sum g^2, #non-finite, flags]`` to a device buffer
before every optimizer step (all-reduced across ranks with the gradient statistics), and the fused
AdamW kernel *skips the update on the device* when the count is non-zero, so the parameters are
protected with no host involvement. With ``EngineConfig.nan_latch`` the count is latched on the
device, so every later step is skipped too until the job halts: the state at exit is the state
before the poisoned step, however far the host has queued ahead.

This trap makes the host aware without a sync in the training loop: after each step the small
report vector (stats + loss) is copied with ``non_blocking=True`` into a pinned (hipHostMalloc)
ring slot on a side stream and an event is recorded. A watcher thread polls the events
(``hipEventQuery``, never a blocking sync), reads the flag and, on a non-finite count, raises a
``divergence`` alert in the :class:`LossSpikeMonitor` and sets :attr:`halted`. The training loop
reads step t's report while the GPU runs step t+1 (:meth:`get`), so every rank takes the halt /
preemption decision for step t at the same loop iteration (the values are all-reduced).
"""
from __future__ import annotations

import threading
import time
from collections import deque
from typing import Callable, Deque, Dict, List, Optional, Tuple

import torch
from ..utils.streams import owned_stream


class NanTrap:
    def __init__(self, device: torch.device, monitor=None, on_trip: Optional[Callable[[int, float], None]] = None,
                 ring: int = 8, poll_s: float = 0.001, width: int = 4):
        self.device = device
        self.monitor = monitor
        self.on_trip = on_trip
        self.halted = False
        self.trip_step: Optional[int] = None
        self.trip_time: Optional[float] = None
        self.records: List[Tuple[int, float, float]] = []  # (step, grad_sumsq, nonfinite)
        self.values: Dict[int, List[float]] = {}  # step -> report vector, until get() takes it
        self.waited = 0  # get() calls that found their step still running on the device (host ran ahead)
        self._cuda = device.type == "cuda"
        self._ring = [torch.zeros(width, dtype=torch.float32, pin_memory=self._cuda) for _ in range(ring)]
        self._slot = 0
        self._pending: Deque = deque()
        self._lock = threading.Lock()
        self._done = threading.Condition(self._lock)
        self._stream = owned_stream(device, "nan-trap", owner=self) if self._cuda else None
        self._stop = threading.Event()
        self._poll_s = poll_s
        self._thread = threading.Thread(target=self._watch, daemon=True, name="nan-trap")
        self._thread.start()

    def record(self, step: int, report: torch.Tensor, issued_at: Optional[float] = None) -> None:
        """Called right after the optimizer step was *queued* (no sync). `report` = [sumsq, nonfinite, ...]."""
        with self._lock:
            full = len(self._pending) >= len(self._ring)
            oldest = self._pending[0][2] if full else None
        if full:  # the host ran a whole ring ahead: wait for the oldest slot to land and be read
            if oldest is not None:
                oldest.synchronize()
            self._wait_drained(len(self._ring) - 1)
        buf = self._ring[self._slot]
        self._slot = (self._slot + 1) % len(self._ring)
        n = min(buf.numel(), report.numel())
        if self._cuda:
            ev = torch.cuda.Event()
            cur = torch.cuda.current_stream(self.device)
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                buf[:n].copy_(report.reshape(-1)[:n], non_blocking=True)
                ev.record(self._stream)
            report.record_stream(self._stream)
        else:
            buf[:n].copy_(report.reshape(-1)[:n])
            ev = None
        with self._lock:
            self._pending.append((step, buf, ev, issued_at or time.time(), n))

    def _wait_drained(self, max_pending: int) -> None:
        with self._done:
            while len(self._pending) > max_pending:
                self._done.wait(self._poll_s * 10)

    def _check(self, step: int, vals: List[float], t_issue: float) -> None:
        ss, bad = vals[0], vals[1]
        self.records.append((step, ss, bad))
        if bad > 0 and not self.halted:
            self.halted = True
            self.trip_step = step
            self.trip_time = time.time()
            if self.monitor is not None:
                self.monitor.ingest_device_stats(step, ss, bad)
            if self.on_trip is not None:
                self.on_trip(step, bad)

    def _watch(self) -> None:
        while not self._stop.is_set():
            item = None
            with self._lock:
                if self._pending:
                    step, buf, ev, t, n = self._pending[0]
                    if ev is None or ev.query():
                        item = (step, buf[:n].tolist(), t)
            if item is None:
                time.sleep(self._poll_s)
                continue
            self._check(item[0], item[1], item[2])
            with self._done:
                self.values[item[0]] = item[1]
                self._pending.popleft()
                self._done.notify_all()

    def get(self, step: int, timeout_s: float = 600.0) -> Optional[List[float]]:
        """Report vector of `step`, waiting for that step to finish on the device (the training loop calls
        this for step t-1 right after queueing step t, so the wait overlaps step t's GPU work)."""
        t0 = time.time()
        ev = None
        with self._lock:
            for s, _, e, _, _ in self._pending:
                if s == step:
                    ev = e
                    break
        if ev is not None:
            if not ev.query():
                self.waited += 1
            ev.synchronize()
        with self._done:
            while step not in self.values:
                if not any(s == step for s, *_ in self._pending):
                    return None  # never recorded
                if time.time() - t0 > timeout_s:
                    raise TimeoutError(f"nan trap: step {step} report not ready after {timeout_s}s")
                self._done.wait(self._poll_s * 10)
            return self.values.pop(step)

    def flush(self, timeout_s: float = 30.0) -> None:
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            with self._lock:
                if not self._pending:
                    return
            time.sleep(self._poll_s)

    def close(self) -> None:
        self.flush()
        self._stop.set()
        self._thread.join(timeout=2)
