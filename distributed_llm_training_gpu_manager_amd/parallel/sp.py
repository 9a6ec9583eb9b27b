"""Sequence parallelism for long context: Ulysses-style head/sequence all-to-all around attention.

SURVEY.md §5.7 asks for a clean context-parallel seam in the attention op; this is the
implementation. Within a sequence-parallel (SP) group of P ranks every rank holds S/P
consecutive tokens of the same sequences. Everything except attention is token-local (norms,
GEMMs, SwiGLU, loss), so only attention needs the whole sequence:

    qkv  [B, S/P, (Hq + 2 Hkv) D]   local tokens, all heads   (RoPE applied with GLOBAL positions)
      -- all-to-all (one call, q/k/v packed) -->
    qkv' [B, S,   (Hq + 2 Hkv)/P D] all tokens, this rank's heads
      flash attention (causal, GQA) on the full sequence  [K6]
    out' [B, S, Hq/P, D] -- all-to-all --> out [B, S/P, Hq, D]

and the exact reverse in the backward (dout in, fused dqkv out). On an 8-GPU MI355X node the
all-to-all is what the point-to-point xGMI mesh serves best (every pair has a direct link; no
ring), and it moves 4 bytes/token/head-dim per direction -- independent of S -- while the
attention work per rank grows with S^2/P. Llama-3-8B (Hkv = 8) supports P up to 8.

The gradient math needs nothing else: SP ranks see different tokens of the same parameters,
exactly like data-parallel ranks, so the ZeRO engine's averaged reduce-scatter over all ranks
already produces the mean over every token of the global batch.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from .comm import Comm


def build_sp_comm(sp_size: int, comm: Optional[Comm] = None) -> Optional[Comm]:
    """Contiguous rank blocks [0..sp-1], [sp..2sp-1], ...; every rank must call this collectively."""
    comm = comm or Comm()
    if sp_size <= 1 or comm.world == 1:
        return None
    world, rank = comm.world, comm.rank
    assert world % sp_size == 0, "world size must be a multiple of sequence_parallel_size"
    mine = None
    for b in range(world // sp_size):
        ranks = list(range(b * sp_size, (b + 1) * sp_size))
        g = comm.new_group(ranks)
        if rank in ranks:
            mine = g
    return mine


def _heads(Hq: int, Hkv: int, P: int) -> Tuple[int, int]:
    assert Hq % P == 0 and Hkv % P == 0, f"heads ({Hq} q, {Hkv} kv) must divide by the SP size {P}"
    return Hq // P, Hkv // P


def _a2a(comm: Comm, send: torch.Tensor) -> torch.Tensor:
    recv = torch.empty_like(send)
    comm.all_to_all_single(recv.view(-1), send.view(-1))
    return recv


def gather_sequence(qkv: torch.Tensor, B: int, S_loc: int, Hq: int, Hkv: int, D: int, comm: Comm) -> torch.Tensor:
    """[B*S_loc, (Hq+2Hkv)D] local tokens -> [B, P*S_loc, hq+2hk, D] full sequence, this rank's heads."""
    P = comm.world
    hq, hk = _heads(Hq, Hkv, P)
    x = qkv.view(B, S_loc, Hq + 2 * Hkv, D)
    q = x[:, :, :Hq].reshape(B, S_loc, P, hq, D)
    k = x[:, :, Hq:Hq + Hkv].reshape(B, S_loc, P, hk, D)
    v = x[:, :, Hq + Hkv:].reshape(B, S_loc, P, hk, D)
    send = torch.cat([q, k, v], dim=3).permute(2, 0, 1, 3, 4).contiguous()  # [P(dst), B, S_loc, hq+2hk, D]
    recv = _a2a(comm, send)  # [P(src = sequence chunk), B, S_loc, hq+2hk, D]
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * S_loc, hq + 2 * hk, D)


def scatter_heads_back(full: torch.Tensor, B: int, S_loc: int, comm: Comm) -> torch.Tensor:
    """[B, P*S_loc, h, D] (this rank's heads) -> [P(src heads), B, S_loc, h, D] for every rank's tokens."""
    P = comm.world
    h, D = full.shape[2], full.shape[3]
    send = full.view(B, P, S_loc, h, D).permute(1, 0, 2, 3, 4).contiguous()  # [P(dst = chunk), B, S_loc, h, D]
    return _a2a(comm, send)


def sp_attention_fwd(qkv: torch.Tensor, B: int, S_loc: int, Hq: int, Hkv: int, D: int, comm: Comm):
    """Causal GQA attention over the whole sequence of an SP group. Returns (out [B, S_loc, Hq, D], saved)."""
    P = comm.world
    hq, hk = _heads(Hq, Hkv, P)
    full = gather_sequence(qkv, B, S_loc, Hq, Hkv, D, comm)
    q, k, v = full[:, :, :hq], full[:, :, hq:hq + hk], full[:, :, hq + hk:]
    o, lse = ops.flash_attn_fwd(q, k, v, causal=True)  # [B, S, hq, D]
    back = scatter_heads_back(o, B, S_loc, comm)  # [P(src heads), B, S_loc, hq, D]
    out = back.permute(1, 2, 0, 3, 4).reshape(B, S_loc, Hq, D)
    return out, (full, o, lse)


def sp_attention_bwd(dout: torch.Tensor, saved, B: int, S_loc: int, Hq: int, Hkv: int, D: int, comm: Comm,
                     dqkv: torch.Tensor) -> torch.Tensor:
    """dout [B, S_loc, Hq, D] -> writes the fused gradient dqkv [B*S_loc, (Hq+2Hkv)D] (local tokens)."""
    full, o, lse = saved
    P = comm.world
    hq, hk = _heads(Hq, Hkv, P)
    send = dout.reshape(B, S_loc, P, hq, D).permute(2, 0, 1, 3, 4).contiguous()
    dfull = _a2a(comm, send).permute(1, 0, 2, 3, 4).reshape(B, P * S_loc, hq, D)
    q, k, v = full[:, :, :hq], full[:, :, hq:hq + hk], full[:, :, hq + hk:]
    dqkv_full = torch.empty(B * P * S_loc, (hq + 2 * hk) * D, dtype=full.dtype, device=full.device)
    ops.flash_attn_bwd(dfull, q, k, v, o, lse, causal=True, dqkv=dqkv_full)
    back = scatter_heads_back(dqkv_full.view(B, P * S_loc, hq + 2 * hk, D), B, S_loc, comm)
    # back: [P(src heads), B, S_loc, hq+2hk, D] -> local rows, heads in global order
    out = dqkv.view(B, S_loc, Hq + 2 * Hkv, D)
    out[:, :, :Hq].view(B, S_loc, P, hq, D).copy_(back[:, :, :, :hq].permute(1, 2, 0, 3, 4))
    out[:, :, Hq:Hq + Hkv].view(B, S_loc, P, hk, D).copy_(back[:, :, :, hq:hq + hk].permute(1, 2, 0, 3, 4))
    out[:, :, Hq + Hkv:].view(B, S_loc, P, hk, D).copy_(back[:, :, :, hq + hk:].permute(1, 2, 0, 3, 4))
    return dqkv
