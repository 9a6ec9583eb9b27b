"""Causal GQA flash attention (kernel: csrc/kernels/flash_attn.hip).

Layout: q ``[B, S, Hq, D]``, k/v ``[B, S, Hkv, D]`` -- strided views straight out
of the fused QKV projection are accepted (unit stride on D only), so the model
never materialises head-major copies. Output ``[B, S, Hq, D]`` contiguous (the
input layout of the output projection GEMM) and the log-sum-exp ``[B, Hq, S]``.

The CPU path is a plain fp32 reference (also used as the numerics oracle).
``backend="sdpa"`` exists only for explicit A/B benchmarking against PyTorch's
own attention; it is never selected implicitly.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .._native import hip_ops, use_native


def _ref_fwd(q, k, v, scale, causal):
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(rep, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)  # [B, Hq, S]
    p = torch.exp(s - lse.unsqueeze(-1))
    o = torch.matmul(p, vf)  # [B, Hq, S, D]
    return o.permute(0, 2, 1, 3).to(q.dtype).contiguous(), lse


def _ref_bwd(dout, q, k, v, out, lse, scale, causal):
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3).repeat_interleave(rep, dim=1)
    vf = v.float().permute(0, 2, 1, 3).repeat_interleave(rep, dim=1)
    do = dout.float().permute(0, 2, 1, 3)
    o = out.float().permute(0, 2, 1, 3)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dv = torch.matmul(p.transpose(-1, -2), do)
    dp = torch.matmul(do, vf.transpose(-1, -2))
    delta = (do * o).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kf)
    dk = torch.matmul(ds.transpose(-1, -2), qf)
    dk = dk.reshape(B, Hkv, rep, S, D).sum(2)
    dv = dv.reshape(B, Hkv, rep, S, D).sum(2)
    t = lambda x: x.permute(0, 2, 1, 3).contiguous()
    return t(dq).to(q.dtype), t(dk).to(k.dtype), t(dv).to(v.dtype)


def flash_attn_fwd(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, softmax_scale: Optional[float] = None,
                   causal: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if use_native(q):
        return hip_ops().flash_attn_fwd(q, k, v, scale, causal)
    return _ref_fwd(q, k, v, scale, causal)


def flash_attn_bwd(dout, q, k, v, out, lse, softmax_scale: Optional[float] = None, causal: bool = True,
                   dqkv: Optional[torch.Tensor] = None):
    """(dq, dk, dv). With ``dqkv`` (contiguous [B*S, (Hq+2Hkv)*D]) the three gradients are written
    straight into that fused buffer (the QKV projection layout) and returned as views of it."""
    scale = softmax_scale if softmax_scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if use_native(q):
        return hip_ops().flash_attn_bwd(dout.contiguous() if dout.stride(-1) != 1 else dout, q, k, v, out, lse,
                                        scale, causal, dqkv)
    dq, dk, dv = _ref_bwd(dout, q, k, v, out, lse, scale, causal)
    if dqkv is None:
        return dq, dk, dv
    B, S = q.shape[:2]
    f = dqkv.view(B, S, -1)
    nq, nk = dq.shape[2] * dq.shape[3], dk.shape[2] * dk.shape[3]
    f[..., :nq].copy_(dq.reshape(B, S, nq))
    f[..., nq:nq + nk].copy_(dk.reshape(B, S, nk))
    f[..., nq + nk:].copy_(dv.reshape(B, S, nk))
    return (f[..., :nq].unflatten(2, dq.shape[2:]), f[..., nq:nq + nk].unflatten(2, dk.shape[2:]),
            f[..., nq + nk:].unflatten(2, dv.shape[2:]))


def sdpa_fwd_bwd_reference(q, k, v, dout, causal=True):
    """PyTorch SDPA forward+backward (A/B benchmark baseline only)."""
    qh = q.permute(0, 2, 1, 3).detach().requires_grad_()
    kh = k.permute(0, 2, 1, 3).detach().requires_grad_()
    vh = v.permute(0, 2, 1, 3).detach().requires_grad_()
    o = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal, enable_gqa=qh.shape[1] != kh.shape[1])
    o.backward(dout.permute(0, 2, 1, 3))
    return o.permute(0, 2, 1, 3), qh.grad.permute(0, 2, 1, 3), kh.grad.permute(0, 2, 1, 3), vh.grad.permute(0, 2, 1, 3)


class FlashAttentionFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        out, lse = flash_attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.causal, ctx.scale = causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        dq, dk, dv = flash_attn_bwd(dout.contiguous(), q, k, v, out, lse, ctx.scale, ctx.causal)
        return dq, dk, dv, None, None


def flash_attention(q, k, v, causal: bool = True, softmax_scale: Optional[float] = None):
    return FlashAttentionFunction.apply(q, k, v, causal, softmax_scale)


def _split_qkv(qkv: torch.Tensor, B: int, S: int, hq: int, hkv: int, d: int):
    f = qkv.view(B, S, -1)
    return (f[..., :hq * d].unflatten(2, (hq, d)), f[..., hq * d:(hq + hkv) * d].unflatten(2, (hkv, d)),
            f[..., (hq + hkv) * d:].unflatten(2, (hkv, d)))


class FlashAttentionQKVFunction(torch.autograd.Function):
    """Attention over a packed QKV projection output [B*S, (Hq+2Hkv)*D]. The backward writes dq/dk/dv
    straight into ONE packed gradient (the layout the QKV GEMM's backward reads), so autograd does
    not build three zero-filled slice gradients and add them up."""

    @staticmethod
    def forward(ctx, qkv, B, S, hq, hkv, d, causal, scale):
        q, k, v = _split_qkv(qkv, B, S, hq, hkv, d)
        out, lse = flash_attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(qkv, out, lse)
        ctx.meta = (B, S, hq, hkv, d, causal, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        B, S, hq, hkv, d, causal, scale = ctx.meta
        q, k, v = _split_qkv(qkv, B, S, hq, hkv, d)
        dqkv = torch.empty(qkv.shape, dtype=qkv.dtype, device=qkv.device)
        flash_attn_bwd(dout.contiguous(), q, k, v, out, lse, scale, causal, dqkv=dqkv)
        return dqkv, None, None, None, None, None, None, None


def flash_attention_qkv(qkv: torch.Tensor, batch: int, seq: int, n_heads: int, n_kv_heads: int, head_dim: int,
                        causal: bool = True, softmax_scale: Optional[float] = None) -> torch.Tensor:
    """out [B, S, Hq, D] = attention(q, k, v) with q|k|v packed per token in a contiguous [B*S, (Hq+2Hkv)*D]."""
    assert qkv.is_contiguous() and qkv.shape == (batch * seq, (n_heads + 2 * n_kv_heads) * head_dim), qkv.shape
    return FlashAttentionQKVFunction.apply(qkv, batch, seq, n_heads, n_kv_heads, head_dim, causal, softmax_scale)
