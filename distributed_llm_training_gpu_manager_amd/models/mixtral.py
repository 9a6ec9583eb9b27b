"""Mixtral 8x7B (sparse MoE, top-2 of 8 experts) with expert parallelism -- BASELINE config 5.

Attention is the Llama block's (GQA, RoPE theta 1e6). The FFN is a routed mixture:

    logits = hn2 @ Wr^T                   [T, E]   (fp32 softmax)
    top-2 per token, gates = softmax over the two selected logits (Mixtral)
    sort (token, k) slots by expert       one-workgroup HIP counting sort (moe_permute), one gather
    EP all-to-all                          rows to the rank owning the expert (RCCL)
    local experts: SwiGLU MLP              grouped MFMA GEMMs, one launch for all experts, group
                                           offsets read on the device (no host sync at EP = 1); the
                                           expert dW deferred to the step's last micro-batch as one
                                           grouped-K launch per weight over K-contiguous operands (the
                                           stashed micro-batches transposed once into an aligned re-layout,
                                           each expert's rows of all micro-batches contiguous)
    EP all-to-all back, combine            out[t] = sum_k gate * y[slot]  (HIP gather kernel)

Backward is hand-written: the combine adjoint gives d(expert outputs) and d(gates),
the expert MLPs run their backward on the expert ranks, the dispatch adjoint is
again a gather-sum (no atomics), and the router gets the top-k softmax gradient
plus the Switch/Mixtral load-balancing auxiliary loss gradient
(coef * E * sum_e f_e * P_e, averaged over layers).

Parameter groups per layer: ``layer{i}`` (attention, norms, router -- ZeRO-sharded
over all ranks) and ``layer{i}.experts`` (this EP rank's experts -- sharded over
the expert-data-parallel group only).
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

import torch

from .. import ops
from ..ops.gemm import grad_mm, transpose_multi
from ..ops import gemm_mfma as gm
from ..ops.moe import moe_combine, moe_combine_bwd, moe_permute, pad_plan_multi
from ..parallel.ep import ExpertDispatcher
from ..utils.streams import side_stream, test_delay
from .common import ParamSpec, Params, StepContext, Unit
from .config import ModelConfig
from .llama import LlamaBlock, LlamaEmbedding, LlamaHead


class MixtralBlock(LlamaBlock):
    def __init__(self, cfg: ModelConfig, layer: int, ep_rank: int = 0, ep_size: int = 1):
        super().__init__(cfg, layer)
        self.ep_rank, self.ep_size = ep_rank, ep_size
        self.E_local = cfg.n_experts // ep_size
        self._dispatcher = None

    def dense_specs(self) -> List[ParamSpec]:
        c = self.cfg
        return [s for s in super().param_specs() if s.name not in ("w_gate_up", "w_down")] + \
            [ParamSpec("router", (c.n_experts, c.d_model), std=c.init_std)]

    def expert_specs(self) -> List[ParamSpec]:
        c = self.cfg
        out_std = c.init_std / (2 * c.n_layers) ** 0.5
        off = self.ep_rank * self.E_local
        # tcache: the engine keeps [E, in, out] transposes (budgeted), so the grouped MFMA dX GEMMs read
        # K-contiguous weights
        tc = True
        return [ParamSpec("w_gate_up", (self.E_local, 2 * c.ffn_dim, c.d_model), std=c.init_std,
                          experts=self.E_local, expert_offset=off, tcache=tc),
                ParamSpec("w_down", (self.E_local, c.d_model, c.ffn_dim), std=out_std,
                          experts=self.E_local, expert_offset=off, tcache=tc)]

    def dispatcher(self, ctx: StepContext):
        if ctx.ep_dispatcher is not None:
            return ctx.ep_dispatcher
        if self._dispatcher is None:
            self._dispatcher = ExpertDispatcher(ctx.ep_group if self.ep_size > 1 else None, self.cfg.n_experts)
        return self._dispatcher

    # ---------------------------------------------------------------- MoE FFN
    def moe_forward(self, p: Params, hn2: torch.Tensor, ctx: StepContext):
        c = self.cfg
        T, E, K = hn2.shape[0], c.n_experts, c.top_k
        probs, topi, gates = ops.router_topk(torch.mm(hn2, p["router"].t()), K)  # [K9]
        offsets, pos, tok = moe_permute(topi, E)  # expert sort on the device, no host read
        counts = (offsets[1:] - offsets[:-1]).long()
        x_sorted = hn2.index_select(0, tok)
        disp = self.dispatcher(ctx)
        x_local, dctx = disp.dispatch(x_sorted, counts, offsets)
        y_local, exp_saved = self._experts_fwd(p, x_local, dctx)
        y_sorted = disp.combine(y_local, dctx)
        out = moe_combine(y_sorted, pos, gates)
        f = counts.float() / float(T * K) * K  # fraction of tokens choosing each expert (summed over k)
        ctx.aux.setdefault("moe_aux", []).append(float(E) * (f * probs.mean(0)).sum())
        return out, (probs, topi, gates, pos, f, x_local, dctx, exp_saved, y_sorted)

    def _grouped(self, x: torch.Tensor) -> bool:
        """Expert GEMMs as single grouped MFMA launches (csrc/kernels/gemm_mfma.hip) with the device
        offsets: no host read of the routing counts, no per-expert launches."""
        c = self.cfg
        return gm.grouped_supported(x) and (2 * c.ffn_dim) % 256 == 0 and c.d_model % 256 == 0 \
            and c.ffn_dim % 256 == 0 and c.d_model % 64 == 0

    def _experts_fwd(self, p: Params, x: torch.Tensor, dctx):
        c = self.cfg
        F = c.ffn_dim
        M = x.shape[0]
        if self._grouped(x):
            offs = dctx.local_offsets
            gu_all = gm.grouped_mm(x, p["w_gate_up"], offs)
            a_all = ops.swiglu_fwd(gu_all, dctx.nrows)  # mesh dispatch: capacity rows, the first nrows valid
            y = gm.grouped_mm(a_all, p["w_down"], offs)
            return y, (gu_all, a_all, dctx)
        counts = dctx.counts()
        gu_all = x.new_empty((M, 2 * F))
        y = x.new_empty((M, c.d_model))
        off = 0
        for e, n in enumerate(counts):
            if n:
                torch.mm(x.narrow(0, off, n), p["w_gate_up"][e].t(), out=gu_all.narrow(0, off, n))
            off += n
        a_all = ops.swiglu_fwd(gu_all)  # the expert segments are contiguous: one launch, no per-expert copy
        off = 0
        for e, n in enumerate(counts):
            if n:
                torch.mm(a_all.narrow(0, off, n), p["w_down"][e].t(), out=y.narrow(0, off, n))
            off += n
        return y, (gu_all, a_all, dctx)

    @staticmethod
    def _grouped_dx(dy: torch.Tensor, p: Params, name: str, offs: torch.Tensor) -> torch.Tensor:
        """dy @ W[e] per expert rows; through the cached [E, in, out] transpose when the engine keeps one."""
        wt = p.get(name + ".T")
        if wt is not None:
            return gm.grouped_mm(dy, wt, offs, transpose_w=True)
        return gm.grouped_mm(dy, p[name], offs, transpose_w=False)

    @staticmethod
    def _expert_dx(dy: torch.Tensor, p: Params, name: str, e: int, out: torch.Tensor) -> None:
        wt = p.get(name + ".T")
        if wt is not None:
            torch.mm(dy, wt[e].t(), out=out)
        else:
            torch.mm(dy, p[name][e], out=out)

    def _experts_bwd(self, p: Params, g: Params, x: torch.Tensor, dy: torch.Tensor, saved, acc: bool, ctx=None):
        gu_all, a_all, dctx = saved
        if self._grouped(x):
            offs = dctx.local_offsets
            dy = dy.contiguous()
            # dA = dY @ W_down fused with the SwiGLU backward in the grouped GEMM's epilogue (dA never stored)
            wt = p.get("w_down.T")
            dgu_all = (gm.grouped_dx_swiglu(dy, wt, offs, gu_all) if wt is not None
                       else gm.grouped_dx_swiglu(dy, p["w_down"], offs, gu_all, transpose_w=False))
            dx = self._grouped_dx(dgu_all, p, "w_gate_up", offs)
            if ctx is not None and ctx.defer_wgrad:
                # dW once per step over the micro-batches' rows regrouped expert-major on the device
                if ctx.micro_index == 0:
                    self._wstash, self._wflushed, self._wbytes = [], False, 0
                # K-major flush: the rows stay row-major until the step's last micro-batch, then
                # each operand of all stashed micro-batches is transposed ONCE into an aligned re-layout where every
                # expert's rows of all micro-batches are contiguous and start on a 64-column boundary -> one plain
                # grouped-K launch per weight (K-contiguous fragments, no per-segment selection in its loop)
                item = (dy, a_all, dgu_all, x, offs)
                self._wstash.append(item)
                self._wbytes += sum(t.numel() * t.element_size() for t in item[:4])
                if ctx.last_micro or self._wbytes > getattr(ctx, "defer_budget_bytes", 48 << 30):
                    self._flush_wgrad_grouped(g, ctx)
                return dx
            xs = self._final_stats(ctx)
            gm.grouped_wgrad(g["w_down"], dy, a_all, offs, acc, stats=xs)
            gm.grouped_wgrad(g["w_gate_up"], dgu_all, x, offs, acc, stats=xs)
            self._count_stats(ctx, xs, 2)
            return dx
        # the per-expert reference path (CPU tensors): reads the routing counts on the host
        counts = dctx.counts()
        if ctx is not None and ctx.defer_wgrad:
            return self._experts_bwd_deferred(p, g, x, dy, saved, counts, ctx)
        dx = torch.empty_like(x)
        da_all = torch.empty_like(a_all)
        off = 0
        for e, n in enumerate(counts):
            if n == 0:
                if not acc:
                    g["w_down"][e].zero_()
                    g["w_gate_up"][e].zero_()
                continue
            dye = dy.narrow(0, off, n)
            grad_mm(g["w_down"][e], dye.t(), a_all.narrow(0, off, n), acc)
            self._expert_dx(dye, p, "w_down", e, da_all.narrow(0, off, n))
            off += n
        dgu_all = ops.swiglu_bwd(da_all, gu_all)  # one launch over every expert's rows
        del da_all
        off = 0
        for e, n in enumerate(counts):
            if n:
                dgu = dgu_all.narrow(0, off, n)
                grad_mm(g["w_gate_up"][e], dgu.t(), x.narrow(0, off, n), acc)
                self._expert_dx(dgu, p, "w_gate_up", e, dx.narrow(0, off, n))
            off += n
        return dx

    def _experts_bwd_deferred(self, p: Params, g: Params, x: torch.Tensor, dy: torch.Tensor, saved, counts,
                              ctx) -> torch.Tensor:
        """Input gradients now, weight gradients once per step: this micro-batch's (dY, A, dGU, X) rows are
        kept and, at the step's last micro-batch (or when the stash budget is reached), every expert's dW is
        ONE GEMM over its rows of all kept micro-batches (K = their token count). Per-expert dW at ~1k
        tokens is bound by the fp32 read-modify-write of the gradient (0.7 GB per expert); concatenating the
        micro-batches pays it once per step (reference: DeepSpeed accumulates per micro-batch)."""
        gu_all, a_all, _ = saved
        if ctx.micro_index == 0:
            self._wstash, self._wflushed, self._wbytes = [], False, 0
        dx = torch.empty_like(x)
        da_all = torch.empty_like(a_all)
        off = 0
        for e, n in enumerate(counts):
            if n:
                self._expert_dx(dy.narrow(0, off, n), p, "w_down", e, da_all.narrow(0, off, n))
            off += n
        dgu_all = ops.swiglu_bwd(da_all, gu_all)
        del da_all
        off = 0
        for e, n in enumerate(counts):
            if n:
                self._expert_dx(dgu_all.narrow(0, off, n), p, "w_gate_up", e, dx.narrow(0, off, n))
            off += n
        self._wstash.append((dy, a_all, dgu_all, x, list(counts)))
        self._wbytes += sum(t.numel() * t.element_size() for t in (dy, a_all, dgu_all, x))
        budget = getattr(ctx, "defer_budget_bytes", 48 << 30)
        if ctx.last_micro or self._wbytes > budget:
            self._flush_wgrad(g)
        return dx

    def _flush_wgrad(self, g: Params) -> None:
        stash, acc = self._wstash, self._wflushed
        for e in range(self.E_local):
            parts = []
            for dy, a, dgu, x, cnt in stash:
                lo, n = sum(cnt[:e]), cnt[e]
                if n:
                    parts.append((dy.narrow(0, lo, n), a.narrow(0, lo, n), dgu.narrow(0, lo, n), x.narrow(0, lo, n)))
            if not parts:
                if not acc:
                    g["w_down"][e].zero_()
                    g["w_gate_up"][e].zero_()
                continue
            cat = (lambda i: parts[0][i]) if len(parts) == 1 else (lambda i: torch.cat([q[i] for q in parts]))
            dye, ae = cat(0), cat(1)
            grad_mm(g["w_down"][e], dye.t(), ae, acc)
            del dye, ae
            dgue, xe = cat(2), cat(3)
            grad_mm(g["w_gate_up"][e], dgue.t(), xe, acc)
            del dgue, xe
        self._wstash, self._wflushed, self._wbytes = [], True, 0

    @staticmethod
    def _final_stats(ctx) -> Optional[torch.Tensor]:
        """The engine's fused expert-statistics accumulator when this launch stores the step's final dW."""
        return ctx.expert_stats if ctx is not None and ctx.last_micro else None

    @staticmethod
    def _count_stats(ctx, xs, n: int) -> None:
        if xs is not None:
            ctx.aux["expert_stats_weights"] = ctx.aux.get("expert_stats_weights", 0) + n

    def _flush_wgrad_grouped(self, g: Params, ctx=None) -> None:
        """Deferred expert dW with device offsets: ONE segmented grouped GEMM per weight reduces each expert over
        its rows of every stashed micro-batch (segment = micro-batch, its offsets row = that micro-batch's
        routing; no host read, no concatenation of the rows)."""
        stash, acc = self._wstash, self._wflushed
        self._wstash, self._wflushed, self._wbytes = [], True, 0
        for i in range(0, len(stash), gm.MAX_SEGMENTS):
            part = stash[i:i + gm.MAX_SEGMENTS]
            offs = torch.stack([t[4] for t in part])  # [segments, experts + 1] int32, on the device
            # the last launch over a weight stores its final gradient: tally the statistics there
            xs = self._final_stats(ctx) if i + gm.MAX_SEGMENTS >= len(stash) else None
            src, poff = pad_plan_multi(offs, sum(int(t[0].shape[0]) for t in part))
            # the w_gate_up operands' re-layout (bandwidth-bound) runs on a side stream under the w_down dW GEMM
            side = side_stream(src.device, "moe_dw")
            cur = torch.cuda.current_stream(src.device) if side is not None else None
            ops_d = (transpose_multi([t[0] for t in part], src), transpose_multi([t[1] for t in part], src))
            if side is not None:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    test_delay()
                    ops_g = (transpose_multi([t[2] for t in part], src), transpose_multi([t[3] for t in part], src))
                ev = torch.cuda.Event()
                ev.record(side)
                for t in part:  # stashed operands freed after the flush: keep them until the side copies ran
                    t[2].record_stream(side)
                    t[3].record_stream(side)
                # the row plan too: allocated on this stream and freed when the flush returns, its block goes straight
                # back to this stream's next allocation. That is ordered today only because this stream waits for
                # the side stream's event below before returning (tests/test_engine_numerics.py scribbles over it)
                src.record_stream(side)
            else:
                ops_g = (transpose_multi([t[2] for t in part], src), transpose_multi([t[3] for t in part], src))
            gm.grouped_wgrad(g["w_down"], ops_d[0], ops_d[1], poff, acc or i > 0, kmajor=True, stats=xs)
            del ops_d
            if side is not None:
                cur.wait_event(ev)
                for t in ops_g:  # allocated on the side stream, consumed here
                    t.record_stream(cur)
            gm.grouped_wgrad(g["w_gate_up"], ops_g[0], ops_g[1], poff, acc or i > 0, kmajor=True, stats=xs)
            del ops_g
            self._count_stats(ctx, xs, 2)

    def moe_backward(self, p: Params, g: Params, hn2: torch.Tensor, saved, dout: torch.Tensor, ctx: StepContext):
        probs, topi, gates, pos, f, x_local, dctx, exp_saved, y_sorted = saved
        disp = self.dispatcher(ctx)
        dy_sorted, dgates = moe_combine_bwd(dout.contiguous(), y_sorted, pos, gates)
        dy_local = disp.redispatch(dy_sorted, dctx)
        dx_local = self._experts_bwd(p, g, x_local, dy_local, exp_saved, ctx.grad_acc, ctx)
        dx_sorted = disp.combine(dx_local, dctx)
        dhn2 = moe_combine(dx_sorted, pos, None)  # adjoint of the dispatch gather: sum the K slots per token
        return self._router_backward(p, g, hn2, probs, topi, gates, f, dgates, dhn2, dout, ctx)

    def _router_backward(self, p: Params, g: Params, hn2, probs, topi, gates, f, dgates, dhn2, dout, ctx):
        c = self.cfg
        T, E = probs.shape
        dtop = gates * (dgates - (gates * dgates).sum(-1, keepdim=True))
        dlogits = torch.zeros(T, E, dtype=torch.float32, device=dout.device).scatter_(1, topi, dtop)
        if c.router_aux_coef > 0:
            # d(coef * mean_l aux_l)/d logits, times the micro-batch share of the loss (grad_scale * tokens)
            scale = c.router_aux_coef * E / (c.n_layers * T) * ctx.grad_scale * ctx.tokens
            daux = scale * probs * (f - (probs * f).sum(-1, keepdim=True))
            dlogits += daux * ctx.loss_scale if ctx.loss_scale is not None else daux
        dl = dlogits.to(hn2.dtype)
        grad_mm(g["router"], dl.t(), hn2, ctx.grad_acc)
        dhn2 = dhn2 + torch.mm(dl, p["router"])
        return dhn2

    # ---------------------------------------------------------------- unit API
    def forward(self, p: Params, x_pair, ctx: StepContext):
        c = self.cfg
        saved_attn, o = self.attn_forward(p, x_pair, ctx)
        x = saved_attn[0]
        hn2, h, rstd2 = ops.rmsnorm_fwd(x, p["mlp_norm"], c.norm_eps, residual=o)
        moe_out, moe_saved = self.moe_forward(p, hn2, ctx)
        return (h, moe_out), (saved_attn, h, rstd2, hn2, moe_saved)

    def backward(self, p: Params, g: Params, saved, dy: torch.Tensor, ctx: StepContext):
        saved_attn, h, rstd2, hn2, moe_saved = saved
        dhn2 = self.moe_backward(p, g, hn2, moe_saved, dy, ctx)
        dh = ops.rmsnorm_bwd(dhn2, h, p["mlp_norm"], rstd2, g["mlp_norm"], dres=dy, accumulate_dw=ctx.grad_acc)
        return self.attn_backward(p, g, saved_attn, dh, ctx)

    def flops(self, ctx: StepContext) -> float:
        c = self.cfg
        T, S = ctx.tokens, ctx.seq_len
        gemm = 2 * T * c.d_model * (c.qkv_dim + c.n_heads * c.head_dim + 3 * c.ffn_dim * c.top_k + c.n_experts)
        return 3.0 * (gemm + 2 * T * S * c.n_heads * c.head_dim)


def build(cfg: ModelConfig, ep_rank: int = 0, ep_size: int = 1):
    """Groups: embed, then per layer (dense, experts), then head. Stages reference (dense, experts)."""
    emb, head = LlamaEmbedding(cfg), LlamaHead(cfg)
    groups: List[Tuple[str, List[ParamSpec], str]] = [("embed", emb.param_specs(), "dense")]
    stages: List[Tuple[Unit, Any]] = [(emb, 0)]
    for i in range(cfg.n_layers):
        blk = MixtralBlock(cfg, i, ep_rank, ep_size)
        groups.append((blk.name, blk.dense_specs(), "dense"))
        groups.append((blk.name + ".experts", blk.expert_specs(), "expert"))
        stages.append((blk, (len(groups) - 2, len(groups) - 1)))
    groups.append(("head", head.param_specs(), "dense"))
    stages.append((head, len(groups) - 1))
    return groups, stages
