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
# Every expert GEMM on the GPU is one grouped MFMA launch with the device offsets (no host read of the routing
# counts, graph-capture safe): forward / dX through the engine's cached [E, in, out] weight transposes, the deferred
# weight gradients as ONE grouped-K launch per weight over K-contiguous operands (the step's micro-batches transposed
# once into an aligned re-layout). Measured alternatives, removed after their A/B (round 3): the per-expert
# hipBLASLt loop that reads the routing counts on the host (125.0k vs 141.8k tok/s, Mixtral-8x7B 2 layers, GA 4),
# the token-major dW kernel, and a static [E, C] capacity layout for batched library GEMMs (100.5k: the random-init
# router overflows the capacity and ~1.1k-row library GEMMs fill 2.2 waves of 256 CUs;
# profiles/moe_experiments_r01.md, README "Measured").


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


def grouped_supported(x: torch.Tensor) -> bool:
    """Can the grouped kernels take rows `x` (bf16, row-major, 16-B aligned, on the GPU with the extension)?"""
    return use_native(x) and _ok(x) and x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0


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


def grouped_dx_swiglu(dy: torch.Tensor, w: torch.Tensor, offsets: torch.Tensor, gu: torch.Tensor,
                      transpose_w: bool = True) -> torch.Tensor:
    """The MoE down projection's input gradient fused with the SwiGLU backward: dA = dy @ w[e]^T per group (as
    grouped_mm), then dgu = swiglu_bwd(dA, gu) -- in the GEMM's epilogue on the GPU, so dA never reaches HBM (a
    [rows, F] write and read saved per micro-batch and layer). gu [R, 2F] (gate | up); returns dgu [R, 2F]. Rows
    outside every group are left unwritten, as swiglu_bwd leaves rows past nrows."""
    if use_native(dy) and os.environ.get("DLGM_MOE_FUSED_SWIGLU", "1") != "0":
        G = w.shape[0]
        N = w.shape[1] if transpose_w else w.shape[2]
        R, K = dy.shape
        out = torch.empty_like(gu)
        b = w.transpose(1, 2) if transpose_w else w
        hip_ops().gemm_mfma(out, dy, b, False, offsets, GROUP_M, R, N, K, G, w.stride(0), None, gu)
        return out
    from .activation import swiglu_bwd
    return swiglu_bwd(grouped_mm(dy, w, offsets, transpose_w), gu)


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
