"""Flat-buffer optimizer primitives (kernel: csrc/kernels/optim.hip).

Everything operates on the ZeRO engine's contiguous per-rank buffers, so each
primitive is one (or two) kernel launches for the whole model partition and
none of them synchronises with the host: clipping and the overflow skip are
decided on the device from the ``stats`` buffer written by :func:`grad_stats`.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .._native import hip_ops, use_native


def grad_stats(grads: Sequence[torch.Tensor], out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """out[0] = sum of squares of finite elements, out[1] = number of non-finite elements."""
    if use_native(out):
        hip_ops().grad_stats(list(grads), out, accumulate)
        return out
    ss = torch.zeros((), dtype=torch.float64, device=out.device)
    bad = torch.zeros((), dtype=torch.float64, device=out.device)
    for g in grads:
        gf = g.detach().float()
        fin = torch.isfinite(gf)
        bad += (~fin).sum()
        ss += torch.where(fin, gf, torch.zeros_like(gf)).double().pow(2).sum()
    if accumulate:
        out[0] += ss.float()
        out[1] += bad.float()
    else:
        out[0] = ss.float()
        out[1] = bad.float()
    return out


def adamw_step_(p: torch.Tensor, m: torch.Tensor, v: torch.Tensor, g: torch.Tensor,
                p16: Optional[torch.Tensor], stats: Optional[torch.Tensor], *, lr: float, beta1: float,
                beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float = 1.0,
                max_norm: float = 0.0, scale_state: Optional[torch.Tensor] = None) -> None:
    """scale_state: the device loss-scaler state [scale, 1/scale, ...]; its 1/scale multiplies grad_scale on
    the device (fp16 path)."""
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if use_native(p):
        hip_ops().adamw_step_(p, m, v, g, p16, stats, lr, beta1, beta2, eps, weight_decay, bc1, bc2,
                              grad_scale, max_norm, scale_state)
        return
    coef = grad_scale * (float(scale_state[1]) if scale_state is not None else 1.0)
    grad_scale = coef
    if stats is not None:
        if float(stats[1]) > 0:
            return
        if max_norm > 0:
            norm = float(stats[0]) ** 0.5 * grad_scale
            coef *= min(1.0, max_norm / (norm + 1e-6))
    gf = g.float() * coef
    p.mul_(1.0 - lr * weight_decay)
    m.mul_(beta1).add_(gf, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if p16 is not None:
        p16.copy_(p.to(p16.dtype))


def accumulate_(dst: torch.Tensor, src: torch.Tensor, alpha: float = 1.0, beta: float = 1.0) -> None:
    """dst(fp32) = beta * dst + alpha * src."""
    if use_native(dst):
        hip_ops().accumulate_(dst, src, alpha, beta)
        return
    if beta == 0.0:
        dst.copy_(src.float() * alpha)
    else:
        dst.mul_(beta).add_(src.float(), alpha=alpha)


def cast_f32_bf16_(dst: torch.Tensor, src: torch.Tensor) -> None:
    if use_native(dst):
        hip_ops().cast_f32_bf16_(dst, src)
        return
    dst.copy_(src.to(dst.dtype))


def loss_scale_update_(state: torch.Tensor, stats: torch.Tensor, window: int, hysteresis: int,
                       min_scale: float) -> None:
    """DeepSpeed dynamic loss-scale update on the device: state = [scale, 1/scale, good steps, hysteresis left],
    stats[1] = non-finite gradient count of the step (no host synchronisation on the GPU)."""
    if use_native(state):
        hip_ops().loss_scale_update_(state, stats, int(window), int(hysteresis), float(min_scale))
        return
    scale, _, good, hyst = (float(x) for x in state[:4].tolist())
    if float(stats[1]) > 0:
        hyst -= 1
        if hyst <= 0:
            scale = max(scale / 2.0, min_scale)
            hyst = hysteresis
        good = 0
    else:
        good += 1
        if good % max(1, window) == 0:
            scale *= 2.0
    state[:4] = torch.tensor([scale, 1.0 / scale, good, hyst], dtype=state.dtype)
