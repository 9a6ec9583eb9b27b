"""Rotary position embedding (rotate-half), applied in place on the fused QKV buffer.

Kernel: ``csrc/kernels/rope.hip``. The cos/sin tables are
built once on the host in fp32 (``[max_pos, head_dim/2]``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import hip_ops, use_native


def rope_tables(head_dim: int, max_pos: int, theta: float, device=None,
                scaling: Optional[dict] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("type") == "llama3":
        # Llama-3.1 frequency scaling (low/high frequency interpolation)
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wavelen = 2 * torch.pi / inv
        smooth = (old / wavelen - lo) / (hi - lo)
        scaled = torch.where(wavelen > old / lo, inv / factor, inv)
        mid = (wavelen <= old / lo) & (wavelen >= old / hi)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv)
    return freqs.cos().float().to(device), freqs.sin().float().to(device)


def rope_(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_rope_heads: int, head_dim: int,
          seq_len: int, inverse: bool = False, pos_ids: Optional[torch.Tensor] = None) -> None:
    """Rotate the first ``n_rope_heads`` heads of every row of ``qkv`` ([T, C]) in place."""
    if use_native(qkv):
        hip_ops().rope_(qkv, cos, sin, pos_ids, n_rope_heads, head_dim, seq_len, inverse)
        return
    T = qkv.shape[0]
    pos = pos_ids if pos_ids is not None else torch.arange(T, device=qkv.device) % seq_len
    c = cos[pos].unsqueeze(1)  # [T, 1, hd/2]
    s = sin[pos].unsqueeze(1)
    if inverse:
        s = -s
    x = qkv[:, : n_rope_heads * head_dim].reshape(T, n_rope_heads, head_dim).float()
    a, b = x[..., : head_dim // 2], x[..., head_dim // 2:]
    out = torch.cat([a * c - b * s, b * c + a * s], dim=-1)
    qkv[:, : n_rope_heads * head_dim].copy_(out.reshape(T, -1).to(qkv.dtype))
