"""Weight-gradient GEMM helper: write or accumulate dW straight into the engine's gradient storage.

On MI355X the gradient partition is fp32 and hipBLASLt runs bf16 x bf16 -> fp32 GEMMs
(``aten::mm.dtype_out`` / ``aten::addmm.dtype_out``) at the speed of the bf16-output
GEMM, so micro-batch gradients are accumulated inside the GEMM epilogue (beta = 1)
instead of being rounded to bf16 and added by a separate pass.
"""
from __future__ import annotations

from typing import Optional

import torch

from .._native import hip_ops, use_native


# hipBLASLt on gfx950, bf16 x bf16 -> fp32 (measured, tools/probe_dw_layout2.py): both operands with
# the reduction (token) dim strided ("NN", what dW = dy^T x is) ~1.0 PF; one operand K-contiguous
# ~1.27 PF; both ~1.35 PF. The HIP transpose streams at ~4.5 TB/s.
_PF = {"NN": 1.0e15, "A": 1.27e15, "B": 1.27e15, "TN": 1.35e15}
_TR_BW, _TR_LAT = 4.5e12, 8e-6


def _tr_cost(t: torch.Tensor) -> float:
    return t.numel() * t.element_size() * 2 / _TR_BW + _TR_LAT


def _plan(a: torch.Tensor, b: torch.Tensor) -> str:
    """Operand layout for out = a @ b with a = dy^T (a view, K strided) and b = x (K strided)."""
    flops = 2.0 * a.shape[0] * a.shape[1] * b.shape[1]
    cost = {"NN": flops / _PF["NN"],
            "A": flops / _PF["A"] + _tr_cost(a),
            "B": flops / _PF["B"] + _tr_cost(b),
            "TN": flops / _PF["TN"] + _tr_cost(a) + _tr_cost(b)}
    return min(cost, key=cost.get)


def grad_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool) -> torch.Tensor:
    """out (+)= a @ b. `out` may be bf16 (scratch, acc must be False) or fp32 (direct accumulation).

    For the weight-gradient shape (a = dy.t() with dy [T, N] row-major, b = x [T, K] row-major) the
    operands whose transpose pays for itself are first made K-contiguous with the HIP transpose.
    """
    if out.is_cuda and a.dtype == torch.bfloat16 and a.dim() == 2 and a.stride(0) == 1 and a.stride(1) != 1 \
            and b.stride(-1) == 1 and a.shape[0] % 8 == 0 and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0:
        plan = _plan(a, b)
        if plan in ("A", "TN"):
            a = transpose(a.t())  # [N, T] contiguous
        if plan in ("B", "TN"):
            b = transpose(b).t()  # [T, K] view of a contiguous [K, T]
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


def transpose(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Contiguous x^T for a 2-D bf16 tensor (register-blocked HIP kernel on the GPU)."""
    if use_native(x) and x.dtype == torch.bfloat16 and x.shape[0] % 8 == 0 and x.shape[1] % 8 == 0 \
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0:
        return hip_ops().transpose(x, out)
    y = x.t().contiguous()
    if out is not None:
        out.copy_(y)
        return out
    return y


def dx_mm(dy: torch.Tensor, p: dict, name: str) -> torch.Tensor:
    """Input gradient dy @ W for a weight stored [out, in]. When the engine supplies the cached
    transpose ``p[name + ".T"]`` ([in, out], refreshed once per optimizer step) the GEMM runs as
    dy @ (W^T)^T -- both operands K-contiguous, hipBLASLt's fastest layout on gfx950."""
    wt = p.get(name + ".T")
    if wt is not None:
        return torch.mm(dy, wt.t())
    return torch.mm(dy, p[name])
