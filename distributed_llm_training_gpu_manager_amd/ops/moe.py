"""MoE ops: router top-k (csrc/kernels/embedding.hip), the device-side expert permute, the gather-based,
deterministic, atomic-free combine and the aligned re-layouts of the deferred expert dW
(csrc/kernels/moe.hip). The reference has no MoE code; its anchor is BASELINE config 5 (Mixtral expert
parallelism) on the reference's 8-GPU preset world (``/root/reference/ai_engine/deepspeed_launcher.py:383-406``)."""
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


def padded_rows(rows: int, groups: int, align: int = 64) -> int:
    """Static upper bound of the aligned re-layout's length (:func:`pad_plan`), a multiple of 8."""
    return (rows + groups * (align - 1) + 7) // 8 * 8


def pad_plan(offsets: torch.Tensor, rows: int, align: int = 64) -> Tuple[torch.Tensor, torch.Tensor]:
    """Aligned re-layout of `rows` expert-sorted rows (offsets int32 [G + 1]): every expert starts on a multiple of
    `align`. Returns (src int32 [padded_rows(rows, G, align)]: padded row -> sorted row or -1, poff int32 [G + 1]:
    the padded offsets, each range a multiple of align). Device-side, no host read."""
    G = offsets.numel() - 1
    P = padded_rows(rows, G, align)
    if use_native(offsets):
        return hip_ops().moe_pad_plan(offsets.contiguous(), P, align)
    off = offsets.long()
    cnt = off[1:] - off[:-1]
    padc = (cnt + align - 1) // align * align
    poff = torch.zeros(G + 1, dtype=torch.long, device=offsets.device)
    poff[1:] = padc.cumsum(0)
    src = torch.full((P,), -1, dtype=torch.int32, device=offsets.device)
    j = torch.arange(rows, device=offsets.device)
    e = torch.bucketize(j, off[1:], right=True)
    src[poff[e] + (j - off[e])] = j.to(torch.int32)
    return src, poff.to(torch.int32)


def pad_plan_multi(offsets: torch.Tensor, rows: int, align: int = 64) -> Tuple[torch.Tensor, torch.Tensor]:
    """:func:`pad_plan` over S row sets at once (offsets int32 [S, G + 1], `rows` = the sets' total): expert e's
    rows of set 0, set 1, ... are contiguous from padded row poff[e] (a multiple of `align`). Returns (src int32
    [padded_rows(rows, G, align)]: (set << 24) | row, or -1; poff int32 [G + 1]). For ops.gemm.transpose_multi."""
    S, G = offsets.shape[0], offsets.shape[1] - 1
    P = padded_rows(rows, G, align)
    if use_native(offsets):
        return hip_ops().moe_pad_plan_multi(offsets.contiguous(), P, align)
    off = offsets.long()
    cnt = off[:, 1:] - off[:, :-1]  # [S, G]
    tot = cnt.sum(0)
    padc = (tot + align - 1) // align * align
    poff = torch.zeros(G + 1, dtype=torch.long)
    poff[1:] = padc.cumsum(0)
    src = torch.full((P,), -1, dtype=torch.int32)
    for e in range(G):
        p = int(poff[e])
        for t in range(S):
            n = int(cnt[t, e])
            lo = int(off[t, e])
            src[p:p + n] = (t << 24) | torch.arange(lo, lo + n, dtype=torch.int32)
            p += n
    return src.to(offsets.device), poff.to(torch.int32).to(offsets.device)


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
