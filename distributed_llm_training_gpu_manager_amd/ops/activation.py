"""SwiGLU on the fused gate/up GEMM output ``gu = [T, 2F]`` (kernel: csrc/kernels/swiglu.hip)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .._native import hip_ops, use_native


def swiglu_fwd(gu: torch.Tensor, nrows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up over gu = [T, 2F]. nrows (int32 [1], device): only the first nrows rows are
    computed on the GPU (the rest is left uninitialised); the CPU reference computes every row."""
    if use_native(gu):
        return hip_ops().swiglu_fwd(gu, nrows)
    f = gu.shape[-1] // 2
    g, u = gu[..., :f].float(), gu[..., f:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(dy: torch.Tensor, gu: torch.Tensor, nrows: Optional[torch.Tensor] = None) -> torch.Tensor:
    if use_native(gu):
        return hip_ops().swiglu_bwd(dy, gu, nrows)
    f = gu.shape[-1] // 2
    g, u, d = gu[..., :f].float(), gu[..., f:].float(), dy.float()
    s = torch.sigmoid(g)
    dg = d * u * (s + g * s * (1 - s))
    du = d * g * s
    return torch.cat([dg, du], dim=-1).to(gu.dtype)
