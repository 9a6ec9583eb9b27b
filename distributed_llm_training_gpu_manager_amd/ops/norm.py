"""RMSNorm (optionally fused with the residual add): HIP kernels on GPU, fp32 reference on CPU.

Kernel: ``csrc/kernels/rmsnorm.hip``. The functional pair
``rmsnorm_fwd`` / ``rmsnorm_bwd`` is what the manual-backward transformer units
call; :class:`RMSNormFunction` wraps it for autograd users.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import hip_ops, use_native


def rmsnorm_fwd(x: torch.Tensor, w: torch.Tensor, eps: float,
                residual: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Return ``(y, h, rstd)`` where ``h = x + residual`` (or ``x``) and ``y = rmsnorm(h) * w``."""
    if use_native(x):
        return hip_ops().rmsnorm_fwd(x, residual, w, eps)
    h = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    hf = h.float()
    rstd = torch.rsqrt(hf.pow(2).mean(-1) + eps)
    y = (hf * rstd.unsqueeze(-1) * w.float()).to(x.dtype)
    return y, h, rstd.reshape(-1)


def rmsnorm_bwd(dy: torch.Tensor, h: torch.Tensor, w: torch.Tensor, rstd: torch.Tensor,
                dw_out: torch.Tensor, dres: Optional[torch.Tensor] = None,
                accumulate_dw: bool = False) -> torch.Tensor:
    """Return dx (+ dres). Writes (or adds) sum_t dy*xhat into ``dw_out``."""
    if use_native(dy):
        return hip_ops().rmsnorm_bwd(dy, h, w, rstd, dres, dw_out, accumulate_dw)
    D = h.shape[-1]
    hf = h.float().reshape(-1, D)
    g = dy.float().reshape(-1, D)
    r = rstd.float().reshape(-1, 1)
    xhat = hf * r
    dw = (g * xhat).sum(0)
    gw = g * w.float()
    dot = (gw * xhat).mean(-1, keepdim=True)
    dx = (gw - xhat * dot) * r
    if dres is not None:
        dx = dx + dres.float().reshape(-1, D)
    if accumulate_dw:
        dw_out.add_(dw.to(dw_out.dtype))
    else:
        dw_out.copy_(dw.to(dw_out.dtype))
    return dx.to(dy.dtype).reshape(dy.shape)


class RMSNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        y, h, rstd = rmsnorm_fwd(x2, w.contiguous(), eps)
        ctx.save_for_backward(h, w, rstd)
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, dy):
        h, w, rstd = ctx.saved_tensors
        dw = torch.empty(w.shape, dtype=torch.float32, device=w.device)
        dx = rmsnorm_bwd(dy.reshape(h.shape).contiguous(), h, w.contiguous(), rstd, dw)
        return dx.reshape(dy.shape), dw.to(w.dtype), None


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    return RMSNormFunction.apply(x, w, eps)


def layernorm_fwd(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float):
    """LayerNorm for the GPT-2 family (autograd units)."""
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)
