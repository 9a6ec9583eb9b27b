"""Fused vocab-parallel-free softmax cross-entropy (kernel: csrc/kernels/cross_entropy.hip).

``cross_entropy_fwd_bwd_`` computes the per-row loss AND overwrites the logits
with ``(softmax - onehot) * grad_scale`` in one kernel: the training engine knows
the loss gradient in advance (1 / tokens), so no second sweep is needed.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import hip_ops, use_native


def cross_entropy_fwd_bwd_(logits: torch.Tensor, labels: torch.Tensor, grad_scale: float,
                           ignore_index: int = -100, compute_grad: bool = True,
                           scale: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Return (loss_per_row fp32 [T], lse fp32 [T]); logits [T, V] become the gradient in place, scaled by
    grad_scale times the optional device word ``scale[0]`` (the fp16 path's dynamic loss scale, read on the
    device: no host synchronisation)."""
    if use_native(logits):
        return hip_ops().cross_entropy_(logits, labels, ignore_index, grad_scale, compute_grad, scale)
    x = logits.float()
    lse = torch.logsumexp(x, dim=-1)
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    picked = x.gather(1, safe.unsqueeze(1)).squeeze(1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    if compute_grad:
        g = torch.softmax(x, dim=-1)
        g.scatter_add_(1, safe.unsqueeze(1), -torch.ones_like(picked).unsqueeze(1))
        g = g * (grad_scale * valid.float()).unsqueeze(1)
        if scale is not None:
            g = g * scale[0].to(g.device)
        logits.copy_(g.to(logits.dtype))
    return loss, lse
