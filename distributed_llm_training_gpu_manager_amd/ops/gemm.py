"""Weight-gradient GEMM helper: write or accumulate dW straight into the engine's gradient storage.

On MI355X the gradient partition is fp32 and hipBLASLt runs bf16 x bf16 -> fp32 GEMMs
(``aten::mm.dtype_out`` / ``aten::addmm.dtype_out``) at the speed of the bf16-output
GEMM, so micro-batch gradients are accumulated inside the GEMM epilogue (beta = 1)
instead of being rounded to bf16 and added by a separate pass.
"""
from __future__ import annotations

import torch


def grad_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool) -> torch.Tensor:
    """out (+)= a @ b. `out` may be bf16 (scratch, acc must be False) or fp32 (direct accumulation)."""
    if out.dtype == a.dtype:
        if acc:
            return torch.addmm(out, a, b, beta=1.0, out=out)
        return torch.mm(a, b, out=out)
    if out.is_cuda:
        if acc:
            return torch.addmm(out, a, b, beta=1.0, out_dtype=out.dtype, out=out)
        return torch.mm(a, b, out_dtype=out.dtype, out=out)
    r = a.float() @ b.float()
    if acc:
        return out.add_(r)
    return out.copy_(r)


def grad_copy(out: torch.Tensor, src: torch.Tensor, acc: bool) -> None:
    if acc:
        out.add_(src.to(out.dtype))
    else:
        out.copy_(src)
