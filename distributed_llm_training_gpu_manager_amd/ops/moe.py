"""MoE ops: router top-k (csrc/kernels/embedding.hip) and the gather-based, deterministic,
atomic-free combine (csrc/kernels/moe.hip)."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import hip_ops, use_native


def router_topk(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """fp32 router logits [T, E] -> (softmax probs [T, E], top-k expert ids [T, k] int64,
    gates [T, k] = softmax over the selected logits) -- Mixtral routing in one pass."""
    logits = logits.float().contiguous()
    if use_native(logits):
        return hip_ops().router_topk(logits, k)
    probs = torch.softmax(logits, dim=-1)
    topv, topi = logits.topk(k, dim=-1)
    return probs, topi, torch.softmax(topv, dim=-1).contiguous()


def moe_permute(topi: torch.Tensor, n_experts: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Expert-sort of the (token, k) slots on the device -> (offsets int32 [E+1], pos [T, K] slot -> sorted
    row, src [T*K] sorted row -> token); stable (token order within an expert), no host sync."""
    topi = topi.contiguous()
    if use_native(topi):
        return hip_ops().moe_permute(topi, n_experts)
    T, K = topi.shape
    flat = topi.reshape(-1)
    order = torch.argsort(flat, stable=True)
    counts = torch.bincount(flat, minlength=n_experts)
    offsets = torch.zeros(n_experts + 1, dtype=torch.int32, device=topi.device)
    offsets[1:] = torch.cumsum(counts, 0).to(torch.int32)
    pos = torch.empty_like(order)
    pos[order] = torch.arange(order.numel(), device=order.device)
    return offsets, pos.view(T, K), torch.div(order, K, rounding_mode="floor")


def moe_combine(y: torch.Tensor, pos: torch.Tensor, gates: Optional[torch.Tensor]) -> torch.Tensor:
    """out[t] = sum_k gates[t,k] * y[pos[t,k]]  (gates=None -> plain sum)."""
    if use_native(y):
        return hip_ops().moe_combine_fwd(y, pos, gates)
    T, K = pos.shape
    rows = y.float()[pos.reshape(-1)].view(T, K, -1)
    if gates is not None:
        rows = rows * gates.float().unsqueeze(-1)
    return rows.sum(1).to(y.dtype)


def moe_combine_bwd(dout: torch.Tensor, y: torch.Tensor, pos: torch.Tensor,
                    gates: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Adjoint of :func:`moe_combine` -> (dy [N, D], dgates [T, K] fp32)."""
    if use_native(y):
        return hip_ops().moe_combine_bwd(dout, y, pos, gates)
    T, K = pos.shape
    d = dout.float()
    dy = torch.zeros_like(y, dtype=torch.float32)
    dy[pos.reshape(-1)] = (d.unsqueeze(1) * gates.float().unsqueeze(-1)).reshape(T * K, -1)
    dg = (d.unsqueeze(1) * y.float()[pos.reshape(-1)].view(T, K, -1)).sum(-1)
    return dy.to(y.dtype), dg
