"""SwiGLU on the fused gate/up GEMM output ``gu = [T, 2F]`` (kernel: csrc/kernels/swiglu.hip)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import hip_ops, use_native


def swiglu_fwd(gu: torch.Tensor) -> torch.Tensor:
    if use_native(gu):
        return hip_ops().swiglu_fwd(gu)
    f = gu.shape[-1] // 2
    g, u = gu[..., :f].float(), gu[..., f:].float()
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(dy: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    if use_native(gu):
        return hip_ops().swiglu_bwd(dy, gu)
    f = gu.shape[-1] // 2
    g, u, d = gu[..., :f].float(), gu[..., f:].float(), dy.float()
    s = torch.sigmoid(g)
    dg = d * u * (s + g * s * (1 - s))
    du = d * g * s
    return torch.cat([dg, du], dim=-1).to(gu.dtype)
