"""On-device NaN/Inf gradient trap (BASELINE config 3).

The engine's ``grad_stats`` kernel writes ``[sum g^2, #non-finite]`` to a device
buffer before every optimizer step, and the fused AdamW kernel already *skips the
update on the device* when the count is non-zero, so the parameters are protected
with no host involvement. This trap makes the host aware without a sync in the
training loop: after each step the 8-byte stats buffer is copied with
``non_blocking=True`` into pinned (hipHostMalloc) memory on a side stream and an
event is recorded; a watcher thread polls the event (``hipEventQuery``, never a
blocking sync), reads the flag and, on a non-finite count, raises a ``divergence``
alert in the :class:`LossSpikeMonitor` and sets :attr:`halted`. The training loop
checks :attr:`halted` at the next step boundary and exits with
``EXIT_NAN_HALT`` so the supervisor can roll back to the last good checkpoint.
Latency to halt: one optimizer step (the poisoned step itself is already skipped).
"""
from __future__ import annotations

import threading
import time
from collections import deque
from typing import Callable, Deque, List, Optional, Tuple

import torch


class NanTrap:
    def __init__(self, device: torch.device, monitor=None, on_trip: Optional[Callable[[int, float], None]] = None,
                 ring: int = 4, poll_s: float = 0.001):
        self.device = device
        self.monitor = monitor
        self.on_trip = on_trip
        self.halted = False
        self.trip_step: Optional[int] = None
        self.trip_time: Optional[float] = None
        self.records: List[Tuple[int, float, float]] = []  # (step, grad_sumsq, nonfinite)
        self._cuda = device.type == "cuda"
        self._ring = [torch.zeros(2, dtype=torch.float32, pin_memory=self._cuda) for _ in range(ring)]
        self._slot = 0
        self._pending: Deque = deque()
        self._lock = threading.Lock()
        self._stream = torch.cuda.Stream(device) if self._cuda else None
        self._stop = threading.Event()
        self._poll_s = poll_s
        self._thread = threading.Thread(target=self._watch, daemon=True, name="nan-trap")
        self._thread.start()

    def record(self, step: int, stats: torch.Tensor, issued_at: Optional[float] = None) -> None:
        """Called right after the optimizer step was *queued* (no sync)."""
        buf = self._ring[self._slot]
        self._slot = (self._slot + 1) % len(self._ring)
        if self._cuda:
            ev = torch.cuda.Event()
            cur = torch.cuda.current_stream(self.device)
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                buf.copy_(stats, non_blocking=True)
                ev.record(self._stream)
        else:
            buf.copy_(stats)
            ev = None
        with self._lock:
            self._pending.append((step, buf, ev, issued_at or time.time()))

    def _check(self, step: int, buf: torch.Tensor, t_issue: float) -> None:
        ss, bad = float(buf[0]), float(buf[1])
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
                    step, buf, ev, t = self._pending[0]
                    if ev is None or ev.query():
                        item = self._pending.popleft()
            if item is None:
                time.sleep(self._poll_s)
                continue
            self._check(item[0], item[1], item[3])

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
