"""Loader for the in-tree native libraries.

``_dlgm_hip.so`` (HIP kernels, registered as ``torch.ops.dlgm.*``) is loaded with
``torch.ops.load_library`` from the package directory -- it is never installed
into site-packages, so a GPU run always executes the kernels built from this tree.

Policy (no silent fallbacks on the GPU): CPU tensors run the PyTorch reference
implementation in :mod:`ops`; a GPU tensor MUST run the HIP kernel, and if the
library is missing or failed to load we raise instead of quietly running an
eager PyTorch path.
"""
from __future__ import annotations

import os
import sys
import threading
from pathlib import Path

import torch

_PKG_DIR = Path(__file__).resolve().parent
# DLGM_HIP_LIB: A/B a different build of the kernels in the same process/device (tools/ab_kernels.sh)
HIP_LIB = Path(os.environ.get("DLGM_HIP_LIB", _PKG_DIR / "_dlgm_hip.so"))
HOST_LIB = _PKG_DIR / "_dlgm_host.so"

_lock = threading.Lock()
_hip_loaded = False
_hip_error: str | None = None


def load_hip() -> bool:
    """Load the HIP kernel library once. Returns True on success."""
    global _hip_loaded, _hip_error
    if _hip_loaded:
        return True
    with _lock:
        if _hip_loaded:
            return True
        if not HIP_LIB.exists():
            _hip_error = f"{HIP_LIB} not built (run `python tools/build_native.py`)"
            return False
        try:
            torch.ops.load_library(str(HIP_LIB))
            _hip_loaded = True
        except Exception as e:  # pragma: no cover - depends on the build
            _hip_error = f"failed to load {HIP_LIB}: {e}"
        return _hip_loaded


def hip_ops():
    """Return ``torch.ops.dlgm``; raises loudly if the kernels are unavailable."""
    if not load_hip():
        raise RuntimeError(
            "MI355X HIP kernels are required for GPU tensors but are unavailable: "
            f"{_hip_error}. Build them with `python tools/build_native.py` (gfx950)."
        )
    return torch.ops.dlgm


def hip_available() -> bool:
    return load_hip()


def use_native(t: torch.Tensor) -> bool:
    """True when `t` lives on the GPU (and therefore must use the HIP kernel). DLGM_FORCE_REFERENCE=1 sends every op
    to its torch reference; a comma list of ops modules (e.g. ``attention,norm``) only those (a diagnostic bisect)."""
    if not t.is_cuda:
        return False
    force = os.environ.get("DLGM_FORCE_REFERENCE", "0")
    if force in ("", "0"):
        return True
    if force == "1":
        return False
    caller = sys._getframe(1).f_globals.get("__name__", "").rsplit(".", 1)[-1]
    return caller not in force.split(",")
