"""Token embedding (kernel: csrc/kernels/embedding.hip).

Forward is a row gather. Backward adds the dY rows into the (fp32) gradient table without
atomics: the token positions are sorted by id once (stable), then each run of equal ids is
summed by one wave in sorted order -- deterministic and free of host synchronisation.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import hip_ops, use_native


def embedding_fwd(table: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """table [V, D], ids (any shape, int64) -> rows [ids.numel(), D]."""
    ids = ids.reshape(-1)
    if use_native(table):
        return hip_ops().embedding_fwd(table, ids.contiguous())
    return F.embedding(ids, table)


def embedding_bwd_(grad: torch.Tensor, dy: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """grad[ids[t]] += dy[t] for every token t (in place; grad may be a view of a flat buffer)."""
    ids = ids.reshape(-1)
    rows = dy.reshape(-1, grad.shape[1])
    if use_native(grad):
        sorted_ids, order = torch.sort(ids, stable=True)
        hip_ops().embedding_bwd_(grad, rows.contiguous(), sorted_ids, order)
        return grad
    grad.index_put_((ids,), rows.to(grad.dtype), accumulate=True)
    return grad
