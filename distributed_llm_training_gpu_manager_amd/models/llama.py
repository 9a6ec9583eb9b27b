"""Llama-3 family (8B / 70B) as explicit-backward units.

Block dataflow per micro-batch (T = B*S tokens, all bf16, fp32 accumulation
inside the kernels):

    x        = xa + xb                (fused into the first RMSNorm; the previous
                                       block hands over its residual as a pair)
    hn1      = rmsnorm(x) * w_attn    [K3]
    qkv      = hn1 @ Wqkv^T           hipBLASLt, one GEMM for q, k and v
    rope_(qkv)                        [K4] in place on the q/k columns
    attn,lse = flash_attn(q, k, v)    [K6] strided views of qkv, causal GQA
    o        = attn @ Wo^T
    hn2, h   = rmsnorm(x + o) * w_mlp [K3, residual add fused]
    gu       = hn2 @ Wgu^T            one GEMM for gate and up ([2F, D])
    a        = silu(g) * u            [K5]
    d        = a @ Wdown^T
    return (h, d)                     the next unit fuses h + d into its norm

Backward is the exact reverse with GEMMs writing dW straight into the flat
gradient buffer (``torch.mm(..., out=view)``). With 288 GB of HBM per MI355X,
all activations of Llama-3-8B at seq 8192 (~1.1 GB/layer) stay resident, so the
default is NO recompute (SURVEY.md §7.2 memory plan).
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

import torch

from .. import ops
from ..ops.gemm import dx_mm, grad_mm, mm
from ..parallel.sp import sp_attention_bwd, sp_attention_fwd
from .common import ParamSpec, Params, StepContext, Unit
from .config import ModelConfig


def _as_pair(x: Any) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    if isinstance(x, tuple):
        return x
    return x, None


class LlamaEmbedding(Unit):
    name = "embed"

    def __init__(self, cfg: ModelConfig):
        self.cfg = cfg

    def param_specs(self) -> List[ParamSpec]:
        return [ParamSpec("tok_embeddings", (self.cfg.vocab_size, self.cfg.d_model), std=self.cfg.init_std,
                          weight_decay=False)]

    def forward(self, p: Params, x, ctx: StepContext):
        ids = ctx.input_ids.reshape(-1)
        return (ops.embedding_fwd(p["tok_embeddings"], ids), None), ids

    def backward(self, p: Params, g: Params, saved, dy, ctx: StepContext):
        ids = saved
        gt = g["tok_embeddings"]
        if not ctx.grad_acc:
            gt.zero_()
        ops.embedding_bwd_(gt, dy, ids)  # sorted-run reduce: no atomics, deterministic [K10]
        return None


class LlamaBlock(Unit):
    def __init__(self, cfg: ModelConfig, layer: int):
        self.cfg = cfg
        self.layer = layer
        self.name = f"layer{layer}"

    def param_specs(self) -> List[ParamSpec]:
        c = self.cfg
        out_std = c.init_std / (2 * c.n_layers) ** 0.5
        return [
            ParamSpec("attn_norm", (c.d_model,), init="ones", weight_decay=False),
            ParamSpec("wqkv", (c.qkv_dim, c.d_model), std=c.init_std, tcache=True),
            ParamSpec("wo", (c.d_model, c.n_heads * c.head_dim), std=out_std, tcache=True),
            ParamSpec("mlp_norm", (c.d_model,), init="ones", weight_decay=False),
            ParamSpec("w_gate_up", (2 * c.ffn_dim, c.d_model), std=c.init_std, tcache=True),
            ParamSpec("w_down", (c.d_model, c.ffn_dim), std=out_std, tcache=True),
        ]

    # -- attention sub-block helpers (shared with Mixtral) --------------------------
    def attn_forward(self, p: Params, x_pair, ctx: StepContext):
        c = self.cfg
        B, S = ctx.batch, ctx.seq_len
        T = B * S
        xa, xb = _as_pair(x_pair)
        hn1, x, rstd1 = ops.rmsnorm_fwd(xa, p["attn_norm"], c.norm_eps, residual=xb)
        qkv = mm(hn1, p["wqkv"].t())
        cos, sin = ctx.rope
        ops.rope_(qkv, cos, sin, c.n_heads + c.n_kv_heads, c.head_dim, S)  # SP: tables start at this chunk
        if ctx.sp_group is not None:
            # sequence parallel: all-to-all to (full sequence, head slice), attention, all-to-all back;
            # the `lse` slot carries what the backward needs
            attn, lse = sp_attention_fwd(qkv, B, S, c.n_heads, c.n_kv_heads, c.head_dim, ctx.sp_group)
        else:
            q, k, v = self._split(qkv, B, S)
            attn, lse = ops.flash_attn_fwd(q, k, v, causal=True)
        attn2d = attn.view(T, c.n_heads * c.head_dim)
        o = mm(attn2d, p["wo"].t())
        return (x, rstd1, hn1, qkv, attn, lse), o

    def _split(self, qkv: torch.Tensor, B: int, S: int):
        c = self.cfg
        hd, H, Hk = c.head_dim, c.n_heads, c.n_kv_heads
        C = qkv.shape[1]
        base = qkv.view(B, S, C)
        q = base[:, :, : H * hd].view(B, S, H, hd)
        k = base[:, :, H * hd:(H + Hk) * hd].view(B, S, Hk, hd)
        v = base[:, :, (H + Hk) * hd:].view(B, S, Hk, hd)
        return q, k, v

    def attn_backward(self, p: Params, g: Params, saved_attn, dh: torch.Tensor, ctx: StepContext):
        """dh: grad wrt h = x + o. Returns dx (including the residual path)."""
        c = self.cfg
        B, S = ctx.batch, ctx.seq_len
        T = B * S
        x, rstd1, hn1, qkv, attn, lse = saved_attn
        attn2d = attn.view(T, c.n_heads * c.head_dim)
        acc = ctx.grad_acc
        grad_mm(g["wo"], dh.t(), attn2d, acc)
        dattn = dx_mm(dh, p, "wo").view_as(attn)
        dqkv = torch.empty_like(qkv).view(T, -1)
        if ctx.sp_group is not None:
            sp_attention_bwd(dattn, lse, B, S, c.n_heads, c.n_kv_heads, c.head_dim, ctx.sp_group, dqkv)
        else:
            q, k, v = self._split(qkv, B, S)
            ops.flash_attn_bwd(dattn, q, k, v, attn, lse, causal=True, dqkv=dqkv)
        cos, sin = ctx.rope
        ops.rope_(dqkv, cos, sin, c.n_heads + c.n_kv_heads, c.head_dim, S, inverse=True)
        grad_mm(g["wqkv"], dqkv.t(), hn1, acc)
        dhn1 = dx_mm(dqkv, p, "wqkv")
        return ops.rmsnorm_bwd(dhn1, x, p["attn_norm"], rstd1, g["attn_norm"], dres=dh, accumulate_dw=acc)

    # -- unit API --------------------------------------------------------------------
    def forward(self, p: Params, x_pair, ctx: StepContext):
        c = self.cfg
        saved_attn, o = self.attn_forward(p, x_pair, ctx)
        x = saved_attn[0]
        hn2, h, rstd2 = ops.rmsnorm_fwd(x, p["mlp_norm"], c.norm_eps, residual=o)
        gu = mm(hn2, p["w_gate_up"].t())
        a = ops.swiglu_fwd(gu)
        d = mm(a, p["w_down"].t())
        return (h, d), (saved_attn, h, rstd2, hn2, gu, a)

    def backward(self, p: Params, g: Params, saved, dy: torch.Tensor, ctx: StepContext):
        c = self.cfg
        saved_attn, h, rstd2, hn2, gu, a = saved
        acc = ctx.grad_acc
        grad_mm(g["w_down"], dy.t(), a, acc)
        da = dx_mm(dy, p, "w_down")
        dgu = ops.swiglu_bwd(da, gu)
        del da
        grad_mm(g["w_gate_up"], dgu.t(), hn2, acc)
        dhn2 = dx_mm(dgu, p, "w_gate_up")
        del dgu
        dh = ops.rmsnorm_bwd(dhn2, h, p["mlp_norm"], rstd2, g["mlp_norm"], dres=dy, accumulate_dw=acc)
        return self.attn_backward(p, g, saved_attn, dh, ctx)

    def flops(self, ctx: StepContext) -> float:
        c = self.cfg
        T, S = ctx.tokens, ctx.seq_len
        gemm = 2 * T * c.d_model * (c.qkv_dim + c.n_heads * c.head_dim + 3 * c.ffn_dim)
        attn = 2 * T * S * c.n_heads * c.head_dim  # causal: half of 4*T*S*D
        return 3.0 * (gemm + attn)


class LlamaHead(Unit):
    """Final RMSNorm + LM head + fused cross-entropy (loss and dlogits in one kernel)."""

    name = "head"

    def __init__(self, cfg: ModelConfig):
        self.cfg = cfg

    def param_specs(self) -> List[ParamSpec]:
        c = self.cfg
        return [ParamSpec("norm", (c.d_model,), init="ones", weight_decay=False),
                ParamSpec("lm_head", (c.vocab_size, c.d_model), std=c.init_std, tcache=True)]

    # [T, V] 16-bit logits above this many bytes are never materialised whole: the forward computes the loss
    # chunk by chunk (CE without gradient) and the backward recomputes each chunk's logits, turns them into
    # dlogits in place and runs that chunk's dX / dW GEMMs (one extra logits GEMM for micro-batches whose
    # logits alone would take more than the budget, e.g. mbs 4 x 8192 tokens x 128k vocab = 8.4 GB)
    logits_budget_bytes = 6 << 30
    chunk_tokens = 8192

    def _chunked(self, T: int) -> bool:
        return T * self.cfg.vocab_size * 2 > self.logits_budget_bytes and T > self.chunk_tokens

    def forward(self, p: Params, x_pair, ctx: StepContext):
        c = self.cfg
        xa, xb = _as_pair(x_pair)
        hn, x, rstd = ops.rmsnorm_fwd(xa, p["norm"], c.norm_eps, residual=xb)
        labels = ctx.labels.reshape(-1)
        T = hn.shape[0]
        if self._chunked(T):
            loss = torch.zeros((), dtype=torch.float32, device=hn.device)
            for lo in range(0, T, self.chunk_tokens):
                n = min(self.chunk_tokens, T - lo)
                logits = mm(hn.narrow(0, lo, n), p["lm_head"].t())
                rows, _ = ops.cross_entropy_fwd_bwd_(logits, labels.narrow(0, lo, n), ctx.grad_scale,
                                                    compute_grad=False)
                loss += rows.sum()
                del logits
            return loss, (x, rstd, hn, None)
        logits = mm(hn, p["lm_head"].t())
        loss_rows, _ = ops.cross_entropy_fwd_bwd_(logits, labels, ctx.grad_scale, scale=ctx.loss_scale)
        # logits now hold d(loss)/d(logits); keep them for backward
        return loss_rows.sum(), (x, rstd, hn, logits)

    def backward(self, p: Params, g: Params, saved, dy, ctx: StepContext):
        x, rstd, hn, dlogits = saved
        if dlogits is None:  # chunked head: recompute each chunk's logits -> dlogits -> its dW / dX share
            labels = ctx.labels.reshape(-1)
            T = hn.shape[0]
            dhn = torch.empty_like(hn)
            for i, lo in enumerate(range(0, T, self.chunk_tokens)):
                n = min(self.chunk_tokens, T - lo)
                hc = hn.narrow(0, lo, n)
                dl = mm(hc, p["lm_head"].t())
                ops.cross_entropy_fwd_bwd_(dl, labels.narrow(0, lo, n), ctx.grad_scale, scale=ctx.loss_scale)
                grad_mm(g["lm_head"], dl.t(), hc, ctx.grad_acc or i > 0)
                dhn.narrow(0, lo, n).copy_(dx_mm(dl, p, "lm_head"))
                del dl
            return ops.rmsnorm_bwd(dhn, x, p["norm"], rstd, g["norm"], accumulate_dw=ctx.grad_acc)
        grad_mm(g["lm_head"], dlogits.t(), hn, ctx.grad_acc)
        dhn = dx_mm(dlogits, p, "lm_head")
        return ops.rmsnorm_bwd(dhn, x, p["norm"], rstd, g["norm"], accumulate_dw=ctx.grad_acc)

    def flops(self, ctx: StepContext) -> float:
        return 3.0 * 2 * ctx.tokens * self.cfg.d_model * self.cfg.vocab_size


def build(cfg: ModelConfig):
    """Return (param_groups, stages); every Llama unit owns exactly one parameter group."""
    units: List[Unit] = [LlamaEmbedding(cfg)] + [LlamaBlock(cfg, i) for i in range(cfg.n_layers)] + [LlamaHead(cfg)]
    groups = [(u.name, u.param_specs()) for u in units]
    return groups, [(u, i) for i, u in enumerate(units)]
