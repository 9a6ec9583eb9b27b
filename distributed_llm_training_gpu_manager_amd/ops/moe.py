"""MoE ops: router top-k (csrc/kernels/embedding.hip), the device-side expert permute, the gather-based,
deterministic, atomic-free combine, the capacity plan and the aligned re-layouts of the deferred expert dW
(csrc/kernels/moe.hip). The reference has no MoE code; its anchor is BASELINE config 5 (Mixtral expert
parallelism) on the reference's 8-GPU preset world (``/root/reference/ai_engine/deepspeed_launcher.py:383-406``)."""
from __future__ import annotations

import math
from dataclasses import dataclass
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


@dataclass
class CapacityPlan:
    """Expert rows laid out for static-shape batched GEMMs (csrc/kernels/moe.hip moe_capacity_plan).

    The expanded row space holds ``G * C`` capacity rows (expert e's first C rows at ``e*C ..``, padding rows
    past the expert's count are zero) followed by ``R`` overflow rows (an expert's rows past its C-th, packed
    expert by expert; ``ovf_offsets`` splits them, ``nrows = G*C + used overflow rows`` on the device).
    Nothing is dropped: the capacity region runs as one batched library GEMM of static shape, the (usually
    empty) overflow region as one grouped launch with device offsets -- no host read of the routing counts.
    """
    G: int
    C: int
    R: int
    exp_src: torch.Tensor      # int32 [G*C + R]: expanded row -> sorted row (-1: padding / unused)
    row_map: torch.Tensor      # int64 [R]: sorted row -> expanded row
    ovf_offsets: torch.Tensor  # int32 [G + 1]: overflow rows per expert (exclusive prefix)
    nrows: torch.Tensor        # int32 [1]: G*C + used overflow rows

    @property
    def gc(self) -> int:
        return self.G * self.C

    @property
    def rows(self) -> int:
        return self.G * self.C + self.R


def capacity_rows(rows: int, groups: int, factor: float, align: int = 64) -> int:
    """Per-expert capacity C for `rows` routed rows over `groups` experts: factor x the balanced share,
    rounded up to `align` rows (at least one aligned block)."""
    c = int(math.ceil(factor * rows / max(1, groups)))
    return max(align, (c + align - 1) // align * align)


def capacity_plan(offsets: torch.Tensor, rows: int, capacity: int) -> CapacityPlan:
    """Build the :class:`CapacityPlan` of `rows` expert-sorted rows split by `offsets` (int32 [G + 1])."""
    G = offsets.numel() - 1
    if use_native(offsets):
        exp_src, row_map, ovf, nrows = hip_ops().moe_capacity_plan(offsets.contiguous(), rows, capacity)
        return CapacityPlan(G, capacity, rows, exp_src, row_map, ovf, nrows)
    off = offsets.long()
    cnt = off[1:] - off[:-1]
    over = (cnt - capacity).clamp(min=0)
    ovf = torch.zeros(G + 1, dtype=torch.long, device=offsets.device)
    ovf[1:] = over.cumsum(0)
    exp_src = torch.full((G * capacity + rows,), -1, dtype=torch.int32, device=offsets.device)
    row_map = torch.empty(rows, dtype=torch.long, device=offsets.device)
    j = torch.arange(rows, device=offsets.device)
    e = torch.bucketize(j, off[1:], right=True)  # expert of each sorted row
    r = j - off[e]
    x = torch.where(r < capacity, e * capacity + r, G * capacity + ovf[e] + (r - capacity))
    exp_src[x] = j.to(torch.int32)
    row_map[:] = x
    nrows = torch.tensor([G * capacity + int(ovf[-1])], dtype=torch.int32, device=offsets.device)
    return CapacityPlan(G, capacity, rows, exp_src, row_map, ovf.to(torch.int32), nrows)


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


def gather_rows(src: torch.Tensor, idx: torch.Tensor, idx2: Optional[torch.Tensor] = None,
                nrows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[r] = src[idx2[idx[r]] if idx2 is given else idx[r]], zero rows where idx[r] < 0 (int32 idx). On the
    GPU rows at or past nrows (int32 [1], device) are left uninitialised."""
    if use_native(src):
        return hip_ops().gather_rows(src.contiguous(), idx, idx2, nrows)
    if src.shape[0] == 0:
        return src.new_zeros((idx.numel(), src.shape[1]))
    s = idx.long()
    valid = s >= 0
    s = s.clamp(min=0)
    if idx2 is not None:
        s = idx2.long()[s]
    out = src.index_select(0, s)
    return out * valid.unsqueeze(1).to(out.dtype)


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
