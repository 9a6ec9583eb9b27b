"""Named side HIP streams for bandwidth-bound work that overlaps the compute stream.

Each (device, name) pair gets one stream for the life of the process. ``side_stream`` returns None on the CPU and
while the current stream is being captured into a HIP graph: captured work stays on the capturing stream (a fork
that a later replay step fails to join would invalidate the capture).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

_STREAMS: Dict[Tuple[int, str], "torch.cuda.Stream"] = {}
TEST_DELAY_CYCLES = {"cycles": 0}  # test hook: side-stream work first spins this long (a missing wait then shows)


def test_delay() -> None:
    """Called at the start of work queued on a side stream (inside its stream context)."""
    if TEST_DELAY_CYCLES["cycles"]:
        torch.cuda._sleep(TEST_DELAY_CYCLES["cycles"])


def side_stream(device: torch.device, name: str) -> Optional["torch.cuda.Stream"]:
    if device.type != "cuda" or torch.cuda.is_current_stream_capturing():
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, name)
    s = _STREAMS.get(key)
    if s is None:
        s = _STREAMS[key] = torch.cuda.Stream(torch.device("cuda", idx))
    return s
