"""Load hipBLASLt/rocBLAS solutions tuned for this framework's GEMM shapes (PyTorch TunableOp).

``tools/tune_gemms.py`` searches every hipBLASLt and rocBLAS solution for the forward and
input-gradient GEMMs of a model at its training token count and writes the winners to
``distributed_llm_training_gpu_manager_amd/tuned/tunableop_<model>_T<tokens>.csv``. Loading
a file turns TunableOp on with tuning OFF: listed shapes use their tuned solution, every other
shape keeps hipBLASLt's default heuristic. Results are keyed by the device / ROCm / hipBLASLt
versions recorded in the file (TunableOp validators), so a file from another stack is ignored.
"""
from __future__ import annotations

import glob
import os
from typing import List, Optional

import torch

TUNED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned")
_loaded: List[str] = []


def tuned_files(model: Optional[str] = None) -> List[str]:
    pat = f"tunableop_{model}_T*.csv" if model else "tunableop_*.csv"
    return sorted(glob.glob(os.path.join(TUNED_DIR, pat)))


def enable_tuned_gemms(model: Optional[str] = None) -> List[str]:
    """Enable TunableOp in read-only mode with the tuned results for `model` (all files if None)."""
    if not torch.cuda.is_available():
        return []
    files = [f for f in tuned_files(model) if f not in _loaded]
    if not files and not _loaded:
        return []
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    for f in files:
        if tun.read_file(f):
            _loaded.append(f)
    return list(_loaded)
