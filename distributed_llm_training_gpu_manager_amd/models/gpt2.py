"""GPT-2 family (BASELINE config 1: GPT-2-small ZeRO-1 plumbing run, CPU/gloo).

Blocks are :class:`AutogradUnit` s that keep their autograd graph from the forward
(LayerNorm / GELU are not on the MI355X headline path); attention still goes through :mod:`ops.attention`, i.e. the HIP
flash kernel on the GPU (head_dim 64 instance) and the fp32 reference on CPU.

Tied input/output embeddings: the embedding table is ONE parameter group that
appears twice in the stage schedule (first as the token/position embedding,
last as the LM head). The engine gathers it at both positions and the two
backward visits accumulate into the same flat gradient segment.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn.functional as F

from .. import ops
from ..ops.gemm import grad_copy, grad_mm, mm
from .common import AutogradUnit, ParamSpec, Params, StepContext, Unit
from .config import ModelConfig


class GPT2Ends:
    """Parameter holder for the tied embedding group (wte, wpe, ln_f)."""

    def __init__(self, cfg: ModelConfig):
        self.cfg = cfg

    def param_specs(self) -> List[ParamSpec]:
        c = self.cfg
        specs = [ParamSpec("wte", (c.vocab_size, c.d_model), std=c.init_std, weight_decay=False),
                 ParamSpec("wpe", (c.max_seq_len, c.d_model), std=0.01, weight_decay=False),
                 ParamSpec("ln_f_w", (c.d_model,), init="ones", weight_decay=False),
                 ParamSpec("ln_f_b", (c.d_model,), init="zeros", weight_decay=False)]
        if not c.tie_embeddings:
            specs.append(ParamSpec("lm_head", (c.vocab_size, c.d_model), std=c.init_std))
        return specs


class GPT2Embed(Unit):
    name = "embed"

    def __init__(self, cfg: ModelConfig):
        self.cfg = cfg

    def forward(self, p: Params, x, ctx: StepContext):
        ids = ctx.input_ids.reshape(-1)
        pos = torch.arange(ctx.seq_len, device=ids.device).repeat(ctx.batch)
        return F.embedding(ids, p["wte"]) + F.embedding(pos, p["wpe"]), (ids, pos)

    def backward(self, p: Params, g: Params, saved, dy, ctx: StepContext):
        ids, pos = saved
        # second backward visit of the tied group: the head already wrote (or added) d(wte) and d(ln_f);
        # ctx.grad_acc is True here, so every write below accumulates
        ops.embedding_bwd_(g["wpe"], dy, pos)
        ops.embedding_bwd_(g["wte"], dy, ids)
        return None


class GPT2Block(AutogradUnit):
    keep_graph = True  # GPT-2-small activations are small: save them instead of re-running the forward

    def __init__(self, cfg: ModelConfig, layer: int):
        self.cfg = cfg
        self.name = f"layer{layer}"

    def param_specs(self) -> List[ParamSpec]:
        c = self.cfg
        D, Fd = c.d_model, c.ffn_dim
        proj_std = c.init_std / (2 * c.n_layers) ** 0.5
        return [
            ParamSpec("ln1_w", (D,), init="ones", weight_decay=False), ParamSpec("ln1_b", (D,), init="zeros", weight_decay=False),
            ParamSpec("attn_w", (3 * D, D), std=c.init_std), ParamSpec("attn_b", (3 * D,), init="zeros", weight_decay=False),
            ParamSpec("proj_w", (D, D), std=proj_std), ParamSpec("proj_b", (D,), init="zeros", weight_decay=False),
            ParamSpec("ln2_w", (D,), init="ones", weight_decay=False), ParamSpec("ln2_b", (D,), init="zeros", weight_decay=False),
            ParamSpec("fc_w", (Fd, D), std=c.init_std), ParamSpec("fc_b", (Fd,), init="zeros", weight_decay=False),
            ParamSpec("out_w", (D, Fd), std=proj_std), ParamSpec("out_b", (D,), init="zeros", weight_decay=False),
        ]

    def fwd(self, p: Params, x: torch.Tensor, ctx: StepContext) -> torch.Tensor:
        c = self.cfg
        B, S, H, hd = ctx.batch, ctx.seq_len, c.n_heads, c.head_dim
        h = F.layer_norm(x, (c.d_model,), p["ln1_w"], p["ln1_b"], c.norm_eps)
        qkv = F.linear(h, p["attn_w"], p["attn_b"])  # [B*S, 3*D]: q | k | v per token
        a = ops.flash_attention_qkv(qkv, B, S, H, H, hd, causal=True)  # one packed dqkv in backward
        x = x + F.linear(a.reshape(B * S, c.d_model), p["proj_w"], p["proj_b"])
        h = F.layer_norm(x, (c.d_model,), p["ln2_w"], p["ln2_b"], c.norm_eps)
        h = F.gelu(F.linear(h, p["fc_w"], p["fc_b"]), approximate="tanh")
        return x + F.linear(h, p["out_w"], p["out_b"])

    def flops(self, ctx: StepContext) -> float:
        c = self.cfg
        T, S = ctx.tokens, ctx.seq_len
        return 3.0 * (2 * T * c.d_model * (4 * c.d_model + 2 * c.ffn_dim) + 2 * T * S * c.d_model)


class GPT2Head(Unit):
    """Final LayerNorm + (tied) LM head + the fused HIP cross-entropy (loss and dlogits in one pass,
    like :class:`~.llama.LlamaHead`): no fp32 logits, no separate softmax forward/backward sweeps."""

    name = "head"

    def __init__(self, cfg: ModelConfig):
        self.cfg = cfg

    def _w(self, p: Params) -> torch.Tensor:
        return p["wte"] if self.cfg.tie_embeddings else p["lm_head"]

    def forward(self, p: Params, x, ctx: StepContext):
        c = self.cfg
        h = F.layer_norm(x, (c.d_model,), p["ln_f_w"], p["ln_f_b"], c.norm_eps).reshape(-1, c.d_model)
        w = self._w(p)
        V = w.shape[0]
        if V % 8:  # the CE kernel wants a 16-byte row stride: logits live in a padded buffer
            logits = torch.empty(h.shape[0], V + (-V) % 8, dtype=h.dtype, device=h.device)[:, :V]
            torch.mm(h, w.t(), out=logits)
        else:
            logits = mm(h, w.t())
        loss_rows, _ = ops.cross_entropy_fwd_bwd_(logits, ctx.labels.reshape(-1), ctx.grad_scale,
                                                   scale=ctx.loss_scale)
        # logits now hold d(loss)/d(logits) (scaled by grad_scale); keep them for backward
        return loss_rows.sum(), (x, logits)

    def backward(self, p: Params, g: Params, saved, dy, ctx: StepContext):
        # first backward visit of the tied group: write (or, under accumulation, add) d(wte) / d(ln_f);
        # the embedding's visit adds later
        c = self.cfg
        x, dlogits = saved
        lw = p["ln_f_w"].detach().requires_grad_(True)
        lb = p["ln_f_b"].detach().requires_grad_(True)
        xin = x.detach().requires_grad_(True)
        with torch.enable_grad():
            h = F.layer_norm(xin, (c.d_model,), lw, lb, c.norm_eps)
        wname = "wte" if c.tie_embeddings else "lm_head"
        grad_mm(g[wname], dlogits.t(), h.detach().reshape(-1, c.d_model), ctx.grad_acc)
        dh = torch.mm(dlogits, self._w(p))
        h.backward(dh.view_as(h))
        for k, leaf in (("ln_f_w", lw), ("ln_f_b", lb)):
            grad_copy(g[k], leaf.grad, ctx.grad_acc)
        if not ctx.grad_acc:
            g["wpe"].zero_()  # the embedding's visit accumulates into it
            if not c.tie_embeddings:
                g["wte"].zero_()
        return xin.grad

    def flops(self, ctx: StepContext) -> float:
        return 3.0 * 2 * ctx.tokens * self.cfg.d_model * self.cfg.vocab_size


def build(cfg: ModelConfig):
    """Return (param_groups, stages): stage = (unit, group index)."""
    ends = GPT2Ends(cfg)
    groups = [("ends", ends.param_specs())]
    stages = [(GPT2Embed(cfg), 0)]
    for i in range(cfg.n_layers):
        blk = GPT2Block(cfg, i)
        groups.append((blk.name, blk.param_specs()))
        stages.append((blk, len(groups) - 1))
    stages.append((GPT2Head(cfg), 0))
    return groups, stages
