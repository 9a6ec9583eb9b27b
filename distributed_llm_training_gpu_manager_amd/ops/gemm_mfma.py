"""Python entry points of the expert-grouped and hand-written MFMA GEMMs.

``mfma_mm(out, a, b, acc)``   out (+)= a @ b for bf16 operand views of any unit-stride layout (gemm_mfma.hip)
``grouped_mm(x, w, offsets)`` expert-grouped forward / input-gradient GEMM (rows split by offsets)
``grouped_wgrad(out, a, b, offsets)`` expert-grouped weight gradient (reduction rows split by offsets)
``grouped_wgrad_segments(out, a_list, b_list, offsets)`` the same over several row sets (micro-batches) at once

The group offsets are an int32 device tensor, so an MoE layer launches its expert GEMMs without
reading the routing counts on the host (graph-capture safe). CPU tensors take an fp32 reference path
(tests).

Two device-offset alternatives were measured this round and dropped (profiles/moe_experiments_r01.md):
hipBLASLt's grouped GEMM with device-side user arguments (hipblaslt_ext::GroupedGemm) fails at run time --
the torch wheel bundles its own libhipblaslt (ROCm 7.0), which the process loads instead of /opt/rocm's 7.2,
and its C++ extension API trips a Tensile "hardware != nullptr" assertion against the 7.2 headers (the C API
used by ops/gemm.py is unaffected); torch._grouped_mm is not capture-safe on this stack ("operation not
permitted when stream is capturing": it synchronises) and ran 117.5k tok/s against the loop's 128.3k.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .._native import hip_ops, use_native

DENSE, GROUP_M, GROUP_K = 0, 1, 2
# Expert GEMM strategy (DLGM_MOE_GROUPED):
#   "1"     (default) every expert GEMM as one grouped MFMA launch with the device offsets: no host read of the
#           routing counts at all (graph-capture safe); the input-gradient GEMMs read the engine's cached
#           [E, in, out] weight transposes, the deferred weight gradients run as ONE segmented launch per weight
#           over the step's micro-batches;
#   "0"     the per-expert hipBLASLt loop: reads the routing counts on the host once per layer and micro-batch;
#   "wgrad" only the weight gradients grouped (MFMA), forward / dX per expert through hipBLASLt.
# Mixtral-8x7B (2 layers, seq 4096, GA 4, one MI355X, round 3): grouped 120.0k tok/s (MFU 0.27) vs loop 125.0k
# (0.29) -- 4 % for no host synchronisation in the micro-batch loop (was 115.1k vs 128.3k before the grouped-M
# tile order, the segmented dW and the expert W^T cache; profiles/moe_experiments_r01.md).
#   "cap"   capacity layout (ops.moe.CapacityPlan): each expert's first C = factor x balanced-share rows as ONE
#           static-shape batched hipBLASLt GEMM per weight (forward, dX, and the deferred dW with K = GA x C), the
#           rows past an expert's capacity as one grouped MFMA launch with device offsets (dropless, no host read);
#           DLGM_MOE_CAPACITY_FACTOR (default 1.125) sets the capacity.
_MODE = os.environ.get("DLGM_MOE_GROUPED", "1")
CAPACITY = _MODE == "cap"
CAPACITY_FACTOR = float(os.environ.get("DLGM_MOE_CAPACITY_FACTOR", "1.125"))
# deferred grouped dW over K-contiguous operands (each stashed micro-batch transposed into an aligned re-layout);
# EP = 1 (one static row count); DLGM_MOE_KMAJOR_DW=0 keeps the token-major (transposed-LDS-read) kernel
KMAJOR_DW = os.environ.get("DLGM_MOE_KMAJOR_DW", "1") != "0"
CAPACITY_ALIGN = 64  # capacity rows per expert are a multiple of this
# the capacity region as ONE torch.bmm per weight (opt-in): on MI355X / this torch build the bf16 batched GEMM at the
# Mixtral-8x7B shape ([8, 1024, 4096] x [8, 4096, 28672]) faulted with an illegal address inside the library
# (gpurun_out probe, round 3), so the default issues one static-shape 2-D GEMM per expert
CAPACITY_BMM = os.environ.get("DLGM_MOE_CAP_BMM", "0") == "1"
GROUPED = _MODE in ("1", "cap")
GROUPED_WGRAD = _MODE in ("1", "wgrad", "cap") and os.environ.get("DLGM_MOE_GROUPED_WGRAD", "1") != "0"


def _ok(t: torch.Tensor) -> bool:
    return t.dtype == torch.bfloat16 and t.data_ptr() % 16 == 0


def supported(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> bool:
    """Can the dense kernel take this problem? (N % 256, K % 64, unit-stride operands, 16-B rows)."""
    if not (use_native(out) and _ok(a) and _ok(b)) or a.dim() != 2 or b.dim() != 2:
        return False
    M, K = a.shape
    N = b.shape[1]
    ak = a.stride(1) == 1
    lda = a.stride(0) if ak else a.stride(1)
    bk = b.stride(0) == 1 and b.stride(1) != 1
    if not bk and b.stride(1) != 1:
        return False
    if not ak and a.stride(0) != 1:
        return False
    ldb = b.stride(1) if bk else b.stride(0)
    return (N % 256 == 0 and K % 64 == 0 and (ak or M % 256 == 0) and lda % 8 == 0 and ldb % 8 == 0
            and out.stride(-1) == 1 and out.stride(0) % 4 == 0 and out.dtype in (torch.float32, torch.bfloat16))


def grouped_supported(x: torch.Tensor, wgrad: bool = False, capacity: bool = False) -> bool:
    """Can the grouped kernels take rows `x` (bf16, row-major, 16-B aligned, on the GPU with the extension)?
    wgrad: asking for the weight-gradient GEMMs only (GROUPED_WGRAD), capacity: for the capacity layout
    (CAPACITY), else for all expert GEMMs (GROUPED)."""
    on = CAPACITY if capacity else GROUPED_WGRAD if wgrad else GROUPED
    return on and use_native(x) and _ok(x) and x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0


def mfma_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool = False) -> torch.Tensor:
    # (a 4-wave, 128x128-per-wave variant of the dense kernel measured 20-30 % slower than these 8 waves on
    # the Llama-3-8B GEMMs -- one barrier per K-tile with one wave per SIMD exposes the DMA and barrier
    # latency, and its 384 live fragment/accumulator registers spill VGPRs into AGPRs;
    # profiles/gemm_mfma_4wave_experiment_r02.log -- and was removed)
    if use_native(out):
        hip_ops().gemm_mfma(out, a, b, acc, None, DENSE, a.shape[0], b.shape[1], a.shape[1], 1, 0)
        return out
    r = a.float() @ b.float()
    return out.add_(r) if acc else out.copy_(r)


def grouped_mm(x: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, transpose_w: bool = True,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[rows of group e] = x[rows of e] @ (w[e]^T if transpose_w else w[e]); x [R, K] row-major,
    w [G, N, K] (transpose_w) or [G, K, N]; offsets int32 [G + 1] on the device."""
    G = w.shape[0]
    N = w.shape[1] if transpose_w else w.shape[2]
    R, K = x.shape
    if out is None:
        out = torch.empty(R, N, dtype=x.dtype, device=x.device)
    if use_native(x):
        b = w.transpose(1, 2) if transpose_w else w
        hip_ops().gemm_mfma(out, x, b, False, offsets, GROUP_M, R, N, K, G, w.stride(0))
        return out
    offs = offsets.tolist()
    for e in range(G):
        lo, hi = offs[e], offs[e + 1]
        if hi > lo:
            we = w[e].t() if transpose_w else w[e]
            out[lo:hi] = (x[lo:hi].float() @ we.float()).to(out.dtype)
    return out


def grouped_wgrad(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, offsets: torch.Tensor,
                  acc: bool = False, kmajor: bool = False, stats: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[e] (+)= a[rows of e]^T @ b[rows of e]: a [R, M], b [R, N] row-major (token rows), out [G, M, N].
    kmajor: a [M, P] and b [N, P] come transposed (K contiguous) with every group's column range a whole number
    of 64-wide tiles, zero padded (ops.moe.pad_plan_multi + ops.gemm.transpose_multi).
    stats: fp32 [>= 2] += [sum of squares of the finite, #non-finite] over the stored out (fp32 out only): the
    native launch tallies them in its epilogue (one partial per tile, summed here in a fixed order), so the
    optimizer's gradient statistics need not re-read the expert gradients (ops.grad_stats semantics)."""
    G, M, N = out.shape
    if use_native(out):
        part = None
        if stats is not None:
            assert out.dtype == torch.float32, "grouped_wgrad: fused statistics need an fp32 out"
            part = torch.empty(2 * G * ((M + 255) // 256) * (N // 256), dtype=torch.float32, device=out.device)
        if kmajor:
            hip_ops().gemm_mfma(out, a, b.t(), acc, offsets, GROUP_K, M, N, a.shape[1], G, 0, part)
        else:
            hip_ops().gemm_mfma(out, a.t(), b, acc, offsets, GROUP_K, M, N, a.shape[0], G, 0, part)
        if part is not None:
            stats[:2] += part.view(-1, 2).sum(0)
        return out
    offs = offsets.tolist()
    for e in range(G):
        lo, hi = offs[e], offs[e + 1]
        if kmajor:
            r = a[:, lo:hi].float() @ b[:, lo:hi].float().t()
        else:
            r = a[lo:hi].float().t() @ b[lo:hi].float()
        if acc:
            out[e].add_(r.to(out.dtype))
        else:
            out[e].copy_(r.to(out.dtype))
    if stats is not None:
        o = out.float()
        fin = torch.isfinite(o)
        stats[0] += torch.where(fin, o, torch.zeros_like(o)).square().sum()
        stats[1] += (~fin).sum().to(stats.dtype)
    return out


def capacity_mm(x: torch.Tensor, w: torch.Tensor, plan, transpose_w: bool = True,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Expert GEMM over a capacity layout (ops.moe.CapacityPlan): the G*C capacity rows as ONE static-shape
    batched GEMM (torch.bmm -> hipBLASLt, either weight layout at library speed), the overflow rows as one
    grouped MFMA launch with the device offsets (its spare blocks exit at once when nothing overflowed).
    x [G*C + R, K] row-major, w [G, N, K] (transpose_w) or [G, K, N]."""
    G, C, gc = plan.G, plan.C, plan.gc
    N = w.shape[1] if transpose_w else w.shape[2]
    if out is None:
        out = torch.empty(x.shape[0], N, dtype=x.dtype, device=x.device)
    wb = w.transpose(1, 2) if transpose_w else w
    xc, oc = x[:gc].view(G, C, x.shape[1]), out[:gc].view(G, C, N)
    if CAPACITY_BMM or not x.is_cuda:
        torch.bmm(xc, wb, out=oc)
    else:  # G static-shape library GEMMs (no host read: the shapes do not depend on the routing)
        for e in range(G):
            torch.mm(xc[e], wb[e], out=oc[e])
    if plan.R > 0:
        grouped_mm(x[gc:], w, plan.ovf_offsets, transpose_w=transpose_w, out=out[gc:])
    return out


def _bmm_f32(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool) -> None:
    """out (+)= a @ b batched, bf16 operands -> fp32 out (hipBLASLt through aten's dtype overloads)."""
    if out.is_cuda:
        if acc:
            torch.baddbmm(out, a, b, out_dtype=torch.float32, out=out)
        else:
            torch.bmm(a, b, out_dtype=torch.float32, out=out)
        return
    r = torch.bmm(a.float(), b.float())
    if acc:
        out.add_(r)
    else:
        out.copy_(r)


def capacity_wgrad(out: torch.Tensor, a: list, b: list, plans: list, acc: bool = False) -> torch.Tensor:
    """out[e] (+)= sum_s a[s][rows of e]^T @ b[s][rows of e] over capacity-layout row sets (one per micro-batch):
    the capacity rows of every set stacked per expert -> ONE batched GEMM with K = sets x C (padding rows are
    zero in a or b, so they add nothing), then the overflow rows as one segmented grouped-K launch (accumulate).
    a[s] [G*C + R_s, M], b[s] [G*C + R_s, N] row-major, out [G, M, N] fp32."""
    G, M, N = out.shape
    C = plans[0].C
    assert all(p.C == C and p.G == G for p in plans)
    gc = G * C
    if len(a) == 1:
        A = a[0][:gc].view(G, C, M)
        B = b[0][:gc].view(G, C, N)
    else:
        A = torch.stack([t[:gc].view(G, C, M) for t in a], dim=1).view(G, len(a) * C, M)
        B = torch.stack([t[:gc].view(G, C, N) for t in b], dim=1).view(G, len(b) * C, N)
    if CAPACITY_BMM or not out.is_cuda:
        _bmm_f32(out, A.transpose(1, 2), B, acc)
    else:
        from .gemm import grad_mm
        for e in range(G):
            grad_mm(out[e], A[e].t(), B[e], acc)
    del A, B
    ovf = [(x[gc:], y[gc:], p.ovf_offsets) for x, y, p in zip(a, b, plans) if p.R > 0]
    for i in range(0, len(ovf), MAX_SEGMENTS):
        part = ovf[i:i + MAX_SEGMENTS]
        grouped_wgrad_segments(out, [t[0] for t in part], [t[1] for t in part], torch.stack([t[2] for t in part]),
                               acc=True)
    return out


MAX_SEGMENTS = 8


def grouped_wgrad_segments(out: torch.Tensor, a: list, b: list, offsets: torch.Tensor,
                           acc: bool = False, kmajor: bool = False) -> torch.Tensor:
    """out[e] (+)= sum_s a[s][rows of e in s]^T @ b[s][rows of e in s]: a[s] [R_s, M], b[s] [R_s, N] row-major,
    offsets [S, G + 1] int32 (row s splits segment s by group), out [G, M, N] fp32. One launch reduces every
    group over its rows of all the segments (the step's micro-batches) without concatenating them.
    kmajor: the operands come transposed, a[s] [M, P], b[s] [N, P] (one P), every group range a multiple of 64
    columns with zero padding (ops.moe.pad_plan + the row-remapped transpose): the K-contiguous kernel."""
    G, M, N = out.shape
    if use_native(out):
        assert len(a) <= MAX_SEGMENTS
        hip_ops().gemm_mfma_seg(out, list(a), list(b), offsets, acc, kmajor)
        return out
    offs = offsets.tolist()
    for e in range(G):
        r = None
        for s, (x, y) in enumerate(zip(a, b)):
            lo, hi = offs[s][e], offs[s][e + 1]
            if kmajor:
                part = x[:, lo:hi].float() @ y[:, lo:hi].float().t()
            else:
                part = x[lo:hi].float().t() @ y[lo:hi].float()
            r = part if r is None else r + part
        if r is None:
            r = torch.zeros(M, N)
        if acc:
            out[e].add_(r.to(out.dtype))
        else:
            out[e].copy_(r.to(out.dtype))
    return out
