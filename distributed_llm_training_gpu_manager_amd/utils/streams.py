"""Named side HIP streams for work that overlaps the compute stream, each a DEDICATED HIP stream.

``torch.cuda.Stream()`` hands out streams from a pool of 32 per priority, round-robin: two logically independent
queues of one process become the same HIP stream once 32 other streams were drawn between them (RCCL's
communicator streams come from that pool too). In the round-4 first-engine mismatch of the Mixtral EP-4
overlapped-optimizer test, the failing engine was the only one whose communicator streams were the HIP streams of
the engine's own W^T-cache and MoE dW re-layout side streams (tools/diag/r05/alias_probe.py forces those aliases on
purpose; see README "Determinism"). Whatever the aliasing exposed, two queues the engine orders with events must not
silently become one queue depending on how many streams the process drew before. So every named stream here is
created with ``hipStreamCreateWithFlags`` (non-blocking) and wrapped as a ``torch.cuda.ExternalStream``: the pool
never hands it to anyone else.

Each (device, name) pair gets one stream for the life of the process. ``side_stream`` returns None on the CPU and
while the current stream is being captured into a HIP graph: captured work stays on the capturing stream (a fork
that a later replay step fails to join would invalidate the capture). ``dedicated_stream`` always returns one (for
owners that manage their own capture rules: communicators, the optimizer stream, the checkpoint copy stream).
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import Dict, Optional, Tuple

import torch

_STREAMS: Dict[Tuple[int, str], "torch.cuda.Stream"] = {}
_KIND_NEXT: Dict[str, int] = {}
_LOCK = threading.Lock()
_HIP = {"lib": None}
_POOL = os.environ.get("DLGM_STREAM_POOL", "0") == "1"  # diagnostic: draw from torch's pool as round 4 did
TEST_DELAY_CYCLES = {"cycles": 0}  # test hook: side-stream work first spins this long (a missing wait then shows)


def test_delay() -> None:
    """Called at the start of work queued on a side stream (inside its stream context)."""
    if TEST_DELAY_CYCLES["cycles"]:
        torch.cuda._sleep(TEST_DELAY_CYCLES["cycles"])


def _hip():
    if _HIP["lib"] is None:
        try:
            lib = ctypes.CDLL("libamdhip64.so")
            lib.hipStreamCreateWithFlags.restype = ctypes.c_int
            lib.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            _HIP["lib"] = lib
        except OSError:
            _HIP["lib"] = False
    return _HIP["lib"]


def _new_stream(idx: int) -> "torch.cuda.Stream":
    if _POOL:
        return torch.cuda.Stream(torch.device("cuda", idx))
    lib = _hip()
    if lib:
        s = ctypes.c_void_p()
        with torch.cuda.device(idx):
            rc = lib.hipStreamCreateWithFlags(ctypes.byref(s), 1)  # hipStreamNonBlocking
        if rc == 0 and s.value:
            return torch.cuda.ExternalStream(s.value, device=torch.device("cuda", idx))
    # no HIP runtime reachable through ctypes: the high-priority pool, which torch / RCCL do not draw from
    return torch.cuda.Stream(torch.device("cuda", idx), priority=-1)


def dedicated_stream(device: torch.device, name: str) -> "torch.cuda.Stream":
    """The process's stream named `name` on `device` (created on first use, never shared with torch's pool)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, name)
    s = _STREAMS.get(key)
    if s is None:
        with _LOCK:
            s = _STREAMS.get(key)
            if s is None:
                s = _STREAMS[key] = _new_stream(idx)
                from .stream_audit import _NAMES
                _NAMES[int(s.cuda_stream)] = name  # reports of the stream audit name the queue
    return s


_FREE: Dict[Tuple[int, str], list] = {}  # (device, kind) -> leased streams whose owner is gone


def _give_back(key: Tuple[int, str], s) -> None:
    with _LOCK:
        _FREE.setdefault(key, []).append(s)


def owned_stream(device: torch.device, kind: str, owner: Optional[object] = None,
                 slots: int = 16) -> "torch.cuda.Stream":
    """A dedicated stream for an object that owns one for its lifetime (a communicator, a mesh, the optimizer /
    checkpoint / NaN-trap copy streams). With `owner`, the stream is LEASED: no other live owner of any kind holds it
    (a free one of this kind is reused, else a new one is created), and it returns to the kind's free list when the
    owner is garbage-collected -- a process that builds thousands of owners (the test suite) creates only as many
    streams as were ever live at once. Without an owner: the next of `slots` round-robin streams of this kind."""
    if _POOL:  # diagnostic A/B only: the round-4 behaviour (a fresh stream from torch's round-robin pool)
        return torch.cuda.Stream(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if owner is None:
        with _LOCK:
            k = _KIND_NEXT.get(kind, 0)
            _KIND_NEXT[kind] = k + 1
        return dedicated_stream(device, f"{kind}#{k % slots}")
    key = (idx, kind)
    with _LOCK:
        free = _FREE.get(key)
        s = free.pop() if free else None
        if s is None:
            k = _KIND_NEXT.get("lease:" + kind, 0)
            _KIND_NEXT["lease:" + kind] = k + 1
    if s is None:
        s = dedicated_stream(device, f"{kind}@{k}")
    weakref.finalize(owner, _give_back, key, s)
    return s


def side_stream(device: torch.device, name: str) -> Optional["torch.cuda.Stream"]:
    if device.type != "cuda" or torch.cuda.is_current_stream_capturing():
        return None
    return dedicated_stream(device, name)
