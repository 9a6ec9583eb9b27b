"""Optional torch.profiler window (ROCm: roctracer/rocprofiler-sdk underneath) -- SURVEY.md §5.1.

The reference only toggles DeepSpeed's ``wall_clock_breakdown``; per-phase HIP-event timers live in
:mod:`utils.timers`. This adds a bounded trace window for kernel-level timelines: wrap N optimizer
steps, then write a Chrome trace (``chrome://tracing`` / Perfetto) per rank. For per-kernel
statistics and hardware counters use ``rocprofv3 --kernel-trace --stats`` / ``--pmc`` instead
(tools/prof_bench.sh, tools/pmc_attn.sh).
"""
from __future__ import annotations

import contextlib
import os
from typing import Iterator, Optional

import torch


@contextlib.contextmanager
def trace_window(out_dir: Optional[str], rank: int = 0, enabled: bool = True) -> Iterator[None]:
    """Record everything inside the block; write ``<out_dir>/trace_rank<r>.json`` at exit."""
    if not enabled or not out_dir:
        yield
        return
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)  # HIP kernels on ROCm
    os.makedirs(out_dir, exist_ok=True)
    with torch.profiler.profile(activities=acts, record_shapes=False, with_stack=False) as prof:
        yield
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    prof.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
