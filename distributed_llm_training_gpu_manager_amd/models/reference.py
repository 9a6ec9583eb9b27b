"""Plain-PyTorch fp32 autograd reference of the Llama / Mixtral units (numerics oracle for tests).

Takes the flat parameter dict produced by ``ZeroEngine.full_params()`` (names
``<group>.<param>``) and returns the mean token loss; ``loss.backward()`` gives
gradients to compare with the engine's hand-written backward.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .config import ModelConfig


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _rope(x, cos, sin):
    # x [B, S, H, hd]; rotate-half
    hd = x.shape[-1]
    a, b = x[..., : hd // 2], x[..., hd // 2:]
    c, s = cos[None, :, None, :], sin[None, :, None, :]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1)


def _attn(q, k, v):
    B, S, H, hd = q.shape
    rep = H // k.shape[2]
    k = k.repeat_interleave(rep, dim=2)
    v = v.repeat_interleave(rep, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / hd ** 0.5
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    p = torch.softmax(s.masked_fill(mask, float("-inf")), dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v)


def moe_ref(x, p, prefix, cfg: ModelConfig):
    """Top-k softmax router (Mixtral: softmax over the selected logits) + SwiGLU experts."""
    E, K, Fd = cfg.n_experts, cfg.top_k, cfg.ffn_dim
    logits = x @ p[prefix + "router"].t()
    topv, topi = logits.topk(K, dim=-1)
    gates = torch.softmax(topv, dim=-1)
    out = torch.zeros_like(x)
    for e in range(E):
        wgu = p[prefix + "experts.w_gate_up"][e]
        wd = p[prefix + "experts.w_down"][e]
        sel = (topi == e)
        rows = sel.any(-1).nonzero().squeeze(-1)
        if rows.numel() == 0:
            continue
        gw = (gates * sel).sum(-1)[rows]
        gu = x[rows] @ wgu.t()
        a = F.silu(gu[:, :Fd]) * gu[:, Fd:]
        out = out.index_add(0, rows, (a @ wd.t()) * gw[:, None])
    return out


def llama_loss(params: Dict[str, torch.Tensor], cfg: ModelConfig, ids: torch.Tensor, labels: torch.Tensor,
               cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    B, S = ids.shape
    H, Hk, hd = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
    x = params["embed.tok_embeddings"][ids.reshape(-1)]
    for i in range(cfg.n_layers):
        pre = f"layer{i}."
        hn = _rms(x, params[pre + "attn_norm"], cfg.norm_eps)
        qkv = (hn @ params[pre + "wqkv"].t()).view(B, S, -1)
        q = qkv[..., : H * hd].view(B, S, H, hd)
        k = qkv[..., H * hd:(H + Hk) * hd].view(B, S, Hk, hd)
        v = qkv[..., (H + Hk) * hd:].view(B, S, Hk, hd)
        q, k = _rope(q, cos[:S], sin[:S]), _rope(k, cos[:S], sin[:S])
        a = _attn(q, k, v).reshape(B * S, H * hd)
        x = x + a @ params[pre + "wo"].t()
        hn = _rms(x, params[pre + "mlp_norm"], cfg.norm_eps)
        if cfg.n_experts:
            x = x + moe_ref(hn, params, pre, cfg)
        else:
            gu = hn @ params[pre + "w_gate_up"].t()
            Fd = cfg.ffn_dim
            x = x + (F.silu(gu[:, :Fd]) * gu[:, Fd:]) @ params[pre + "w_down"].t()
    hn = _rms(x, params["head.norm"], cfg.norm_eps)
    logits = hn @ params["head.lm_head"].t()
    return F.cross_entropy(logits.float(), labels.reshape(-1))


def gpt2_loss(params: Dict[str, torch.Tensor], cfg: ModelConfig, ids: torch.Tensor,
              labels: torch.Tensor) -> torch.Tensor:
    """Plain fp32 GPT-2 (pre-LN, GELU-tanh, tied or untied LM head) for the engine's numerics tests."""
    B, S = ids.shape
    H, D = cfg.n_heads, cfg.d_model
    hd = D // H
    pos = torch.arange(S).repeat(B)
    x = params["ends.wte"][ids.reshape(-1)] + params["ends.wpe"][pos]
    for i in range(cfg.n_layers):
        pre = f"layer{i}."
        h = F.layer_norm(x, (D,), params[pre + "ln1_w"], params[pre + "ln1_b"], cfg.norm_eps)
        qkv = (h @ params[pre + "attn_w"].t() + params[pre + "attn_b"]).view(B, S, 3, H, hd)
        a = _attn(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]).reshape(B * S, D)
        x = x + a @ params[pre + "proj_w"].t() + params[pre + "proj_b"]
        h = F.layer_norm(x, (D,), params[pre + "ln2_w"], params[pre + "ln2_b"], cfg.norm_eps)
        h = F.gelu(h @ params[pre + "fc_w"].t() + params[pre + "fc_b"], approximate="tanh")
        x = x + h @ params[pre + "out_w"].t() + params[pre + "out_b"]
    h = F.layer_norm(x, (D,), params["ends.ln_f_w"], params["ends.ln_f_b"], cfg.norm_eps)
    w = params["ends.wte"] if cfg.tie_embeddings else params["ends.lm_head"]
    return F.cross_entropy((h @ w.t()).float(), labels.reshape(-1))
