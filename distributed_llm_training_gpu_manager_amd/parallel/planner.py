"""Per-rank HBM planner: what one rank of a world-W ZeRO job holds on its MI355X (288 GB HBM3E).

VERDICT r1 item 1c: prove, without an 8-GPU box, that BASELINE configs 3-5 (Llama-3-8B and
Llama-3-70B ZeRO-3, Mixtral-8x7B with EP=8, all at W=8) fit. The planner mirrors the engine's
own allocation decisions instead of a rule of thumb:

* the flat groups are built from the model's real parameter specs (``ZeroEngine`` does the same),
  so shard sizes include the ALIGN x W padding and the expert groups' expert-data-parallel sharding;
* ``local_grad_accum``, ``stage3_max_live_parameters`` / ``max_reuse_distance`` ("hbm") and the
  transposed-weight cache budget are resolved with the engine's rules (``ZeroEngine._want_local_grads``,
  ``ResidencyPlan``, ``_add_resident_tcache``);
* activations follow the units' saved tuples (``models/llama.py`` ``forward`` returns, Mixtral's MoE
  saved rows at balanced routing), with and without activation checkpointing.

It is calibrated against measured peaks (``profiles/shadow_rank_*.json``: the shadow-rank runs on one
MI355X, ``parallel.comm.ShadowComm``) and the 1-GPU headline bench; tests/test_planner.py pins both.
The reference has no memory planning at all -- DeepSpeed's ``offload_param`` / ``offload_optimizer``
presets (``ai_engine/deepspeed_launcher.py:383-406``) are its only answer to a model that does not fit.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..models import ModelConfig, build_model

GiB = 1024 ** 3
MI355X_HBM = int(287.98 * GiB)  # bytes: what torch.cuda.get_device_properties reports for one MI355X


@dataclass
class RankPlan:
    model: str
    world: int
    zero_stage: int
    ep_size: int
    parts: Dict[str, float] = field(default_factory=dict)  # bytes
    notes: List[str] = field(default_factory=list)
    hbm_bytes: float = MI355X_HBM

    @property
    def total(self) -> float:
        return sum(self.parts.values())

    @property
    def headroom(self) -> float:
        return 1.0 - self.total / self.hbm_bytes

    def fits(self, min_headroom: float = 0.10) -> bool:
        return self.headroom >= min_headroom

    def summary(self) -> Dict[str, object]:
        return {"model": self.model, "world": self.world, "zero_stage": self.zero_stage, "ep_size": self.ep_size,
                "total_GiB": round(self.total / GiB, 2), "hbm_GiB": round(self.hbm_bytes / GiB, 2),
                "headroom": round(self.headroom, 4),
                "parts_GiB": {k: round(v / GiB, 2) for k, v in self.parts.items()}, "notes": self.notes}


def _activation_bytes(m: ModelConfig, tokens: int, seq: int, ckpt: bool, ep_size: int) -> Dict[str, float]:
    """Saved activations of one micro-batch + the transient peak of one unit's backward."""
    T, D = tokens, m.d_model
    bf = 2
    if m.arch == "gpt2":
        per_layer = bf * T * (9 * D + 2 * m.ffn_dim) + 4 * T * (2 + m.n_heads)
        transient = bf * T * (2 * m.ffn_dim + 3 * D)
    else:
        attn_part = bf * T * (4 * D + m.qkv_dim + m.n_heads * m.head_dim) + 4 * T * (2 + m.n_heads)
        if m.n_experts:
            R = T * m.top_k  # rows this rank's experts process at balanced routing (any EP size)
            moe = bf * R * (2 * D + 3 * m.ffn_dim) + T * (4 * m.n_experts + 16 * m.top_k + 4 * m.top_k)
            per_layer = attn_part + moe + bf * T * D
            transient = bf * R * (3 * m.ffn_dim + 2 * D)
        else:
            per_layer = attn_part + bf * T * 3 * m.ffn_dim
            transient = bf * T * (3 * m.ffn_dim + 2 * D)
    L = m.n_layers
    head = bf * T * (2 * D + m.vocab_size) + 4 * T * 2
    if ckpt:
        saved = L * 2 * bf * T * D  # each unit keeps its input pair (h, d)
        live = per_layer  # one unit recomputed at a time
    else:
        saved, live = L * per_layer, 0.0
    return {"activations_saved": saved + bf * T * D, "activations_recompute": live,
            "backward_transient": transient, "logits": head}


def runtime_reserve(other_bytes: float) -> float:
    """hipBLASLt workspaces, RCCL channel buffers, the caching allocator's rounding and fragmentation.
    Calibrated on the 1-GPU Llama-3-8B bench (planned 185 GiB of tensors vs 185.1 GiB measured peak)."""
    return 2.0 * GiB + 0.03 * other_bytes


def zero3_budgets(hbm_bytes: float, committed_bytes: float, live_hbm_fraction: float = 0.12,
                  tcache_hbm_fraction: float = 0.08, headroom: float = 0.10):
    """'hbm' sizing of the two optional ZeRO-3 HBM consumers, shared by the engine and the planner.

    ``committed_bytes``: everything else the rank will hold at its peak (persistent shards, local
    gradients, activations, reduce scratch, in-flight gathers, runtime reserve). What is left under
    (1 - headroom) of the device goes first to gathered units kept resident across visits (fewer
    all-gathers), then to their transposed-weight caches (faster dX GEMMs), each capped by its
    fraction of HBM. Returns (max_live_parameters in elements, transposed-cache budget in bytes
    given the resident bytes actually used)."""
    avail = max(0.0, (1.0 - headroom) * hbm_bytes - committed_bytes)
    live_bytes = min(live_hbm_fraction * hbm_bytes, avail)

    def tcache_budget(resident_bytes: float) -> float:
        return min(tcache_hbm_fraction * hbm_bytes, max(0.0, avail - resident_bytes))
    return live_bytes / 2.0, tcache_budget


def snapshot_bytes(m: ModelConfig, *, world: int, zero_stage: int = 3, ep_size: int = 1) -> int:
    """Bytes of one rank's checkpoint snapshot (ckpt/checkpoint.py: fp32 master | exp_avg | exp_avg_sq | 16-bit
    params = 14 B per element of the rank's partition), from the same group layout the engine builds; the largest
    rank (shards differ by at most one padding unit) plus 64 MiB of slack."""
    from .zero import FlatGroup

    ep = max(1, ep_size) if m.n_experts else 1
    P = 1 if zero_stage == 0 else world
    groups_spec, _ = build_model(m, 0, ep)
    shard = 0
    for i, grp in enumerate(groups_spec):
        kind = grp[2] if len(grp) > 2 else "dense"
        Pg = (1 if zero_stage == 0 else world // ep) if kind == "expert" else P
        shard += FlatGroup(i, grp[0], grp[1], Pg, kind).shard_numel
    return int(14 * shard + (64 << 20))


def plan_rank(m: ModelConfig, *, world: int, zero_stage: int = 3, micro_batch: int = 1, seq_len: int = 8192,
              grad_accum: int = 8, activation_checkpointing: bool = False, ep_size: int = 1,
              local_grad_accum="hbm", local_grad_hbm_fraction: float = 0.15, max_live_parameters="hbm",
              max_reuse_distance="hbm", live_hbm_fraction: float = 0.12, prefetch_bucket_size: float = 5e8,
              transposed_weight_cache: bool = True, tcache_hbm_fraction: float = 0.08,
              expert_weight_cache: bool = True,
              defer_expert_wgrad="auto", defer_wgrad_budget_gb: float = 48.0,
              offload_optimizer: str = "none", offload_param: str = "none",
              hbm_bytes: float = MI355X_HBM, headroom: float = 0.10) -> RankPlan:
    from .residency import ResidencyPlan, resolve_limit
    from .zero import FlatGroup

    ep = max(1, ep_size) if m.n_experts else 1
    if world % ep:
        raise ValueError("world must be a multiple of the EP size")
    P = 1 if zero_stage == 0 else world
    groups_spec, stages = build_model(m, 0, ep)
    groups: List[FlatGroup] = []
    for i, grp in enumerate(groups_spec):
        kind = grp[2] if len(grp) > 2 else "dense"
        Pg = (1 if zero_stage == 0 else world // ep) if kind == "expert" else P
        groups.append(FlatGroup(i, grp[0], grp[1], Pg, kind))
    shard = sum(g.shard_numel for g in groups)
    full = sum(g.numel for g in groups)
    red_full = sum(g.numel for g in groups if g.P > 1)
    plan = RankPlan(m.name, world, zero_stage, ep, hbm_bytes=hbm_bytes)
    parts = plan.parts
    host_opt = offload_optimizer in ("cpu", "nvme")
    host_par = zero_stage == 3 and offload_param in ("cpu", "nvme")
    parts["fp32_master_m_v"] = 0.0 if host_opt else 12.0 * shard
    parts["fp32_grad_shard"] = 4.0 * shard
    parts["bf16_param_shard"] = 0.0 if host_par else 2.0 * shard
    if host_opt:
        plan.notes.append(f"optimizer state on {offload_optimizer}: {12.0 * shard / GiB:.1f} GiB host")
    if zero_stage in (1, 2):
        parts["bf16_params_full"] = 2.0 * full
    # local fp32 gradient accumulation (ZeroEngine._want_local_grads)
    local = False
    if zero_stage in (2, 3) and red_full:
        if isinstance(local_grad_accum, str):
            local = grad_accum > 1 and 4 * red_full <= local_grad_hbm_fraction * hbm_bytes
        else:
            local = bool(local_grad_accum)
    if zero_stage == 1 or local:
        parts["fp32_grad_full"] = 4.0 * red_full
    # gradient reduce-scatter scratch: bf16 segment + its shard output, two units in flight
    if zero_stage in (2, 3) and red_full:
        big = max(g.numel for g in groups if g.P > 1)
        parts["grad_reduce_scratch"] = 2.0 * 2 * big * (1 + 1.0 / world)
    parts.update(_activation_bytes(m, micro_batch * seq_len, seq_len, activation_checkpointing, ep))
    direct = zero_stage in (0, 1) or local or world == 1
    if m.n_experts and grad_accum > 1 and direct and defer_expert_wgrad in ("auto", True):
        # deferred expert dW (models/mixtral.py): (dY, A, dGU, X) rows of earlier micro-batches, capped
        # + the flush transients (the current micro-batch's rows held to the flush, the per-expert
        # concatenations): 0.45 of one micro-batch's stash, calibrated on the Mixtral EP=8 shadow rank
        R = micro_batch * seq_len * m.top_k
        per = 2.0 * R * (2 * m.d_model + 3 * m.ffn_dim) * m.n_layers
        parts["moe_wgrad_stash"] = min((grad_accum - 1) * per, defer_wgrad_budget_gb * GiB) + 0.45 * per
    st = [tuple(gi) if isinstance(gi, (tuple, list)) else (gi,) for _, gi in stages]
    gathered = [zero_stage == 3 and g.P > 1 for g in groups]
    stage_sz = [sum(groups[gi].numel for gi in s if gathered[gi]) for s in st]
    if zero_stage == 3:
        # current stage + one prefetched stage (stage3_prefetch_bucket_size below one block)
        top = sorted(stage_sz, reverse=True)
        parts["bf16_gathered_inflight"] = 2.0 * (top[0] + (top[1] if len(top) > 1 else 0))
    if host_par:
        parts["offload_param_staging"] = 2.0 * 2 * max(g.shard_numel for g in groups)
        if offload_param == "nvme":  # the partition is a file; host RAM holds the AIO ring (5 group shards)
            plan.notes.append(f"parameters on nvme: {2.0 * shard / GiB:.1f} GiB file, "
                              f"{5 * 2.0 * max(g.shard_numel for g in groups) / GiB:.1f} GiB pinned ring")
        else:
            plan.notes.append(f"parameters on {offload_param}: {2.0 * shard / GiB:.1f} GiB host")
    parts["runtime_reserve"] = runtime_reserve(sum(parts.values()))
    tc_names = lambda g: [sp for sp in g.specs if sp.tcache and len(sp.shape) == 2]  # noqa: E731
    # expert-stacked [E, out, in] weights of groups that are never gathered (ZeroEngine.__init__: within
    # tcache_hbm_fraction of the device, in group order)
    stacked, sused = 0.0, 0.0
    if transposed_weight_cache and expert_weight_cache:
        for g in groups:
            if zero_stage < 3 or g.P == 1:
                nb = 2.0 * sum(sp.numel for sp in g.specs if sp.tcache and len(sp.shape) == 3)
                if nb and sused + nb <= tcache_hbm_fraction * hbm_bytes:
                    sused += nb
        stacked = sused
    if zero_stage == 3 and not host_par:
        committed = sum(parts.values())
        live_params, tc_budget = zero3_budgets(hbm_bytes, committed, live_hbm_fraction, tcache_hbm_fraction,
                                               headroom)
        visits = st + st[::-1]
        rp = ResidencyPlan(visits, [g.numel for g in groups], gathered,
                           resolve_limit(max_live_parameters, lambda: live_params),
                           resolve_limit(max_reuse_distance, lambda: live_params, unbounded_for_hbm=True))
        parts["bf16_gathered_resident"] = 2.0 * rp.resident_params
        tc = 0.0
        if transposed_weight_cache:
            budget = tc_budget(2.0 * rp.resident_params)
            for g in groups:
                nb = 2.0 * sum(sp.numel for sp in tc_names(g))
                if nb and g.P == 1:
                    tc += nb
            used = 0.0
            for g in groups:
                nb = 2.0 * sum(sp.numel for sp in tc_names(g))
                if nb and g.P > 1 and rp.held_through_step(g.idx) and used + nb <= budget:
                    used += nb
            tc += used
        parts["bf16_weight_T_cache"] = tc + stacked
    elif transposed_weight_cache and zero_stage < 3:
        parts["bf16_weight_T_cache"] = 2.0 * sum(sp.numel for g in groups for sp in tc_names(g)) + stacked
    return plan


@dataclass
class MicroBatchChoice:
    micro_batch: int
    grad_accum: int
    activation_checkpointing: bool
    plan: RankPlan
    tried: List[Dict[str, object]] = field(default_factory=list)

    def summary(self) -> Dict[str, object]:
        return {"micro_batch": self.micro_batch, "grad_accum": self.grad_accum,
                "activation_checkpointing": self.activation_checkpointing,
                "total_GiB": round(self.plan.total / GiB, 2), "headroom": round(self.plan.headroom, 4),
                "tried": self.tried}


def auto_micro_batch(m: ModelConfig, *, world: int, seq_len: int, global_batch: Optional[int] = None,
                     grad_accum: int = 8, max_micro: int = 64, allow_checkpointing: bool = True,
                     force_checkpointing: bool = False, min_headroom: float = 0.10,
                     data_parallel: Optional[int] = None, **plan_kw) -> MicroBatchChoice:
    """Micro-batch auto-sizing from the per-rank HBM plan (the reference's launcher docstring claims
    "automatic micro-batch sizing", ``ai_engine/deepspeed_launcher.py:7-8``, and never implements it --
    SURVEY A23).

    Largest micro-batch (sequences per rank per micro-step) whose plan keeps ``min_headroom`` of the
    GPU free, preferring no activation checkpointing (recompute costs ~1/3 of the forward) over a larger
    micro-batch with it. With ``global_batch`` (sequences per optimizer step over the data-parallel
    ranks; EP and ZeRO shard inside the same world) only micro-batches that divide it are tried and the
    gradient accumulation follows; without it the tokens per step are kept: GA = grad_accum / mbs.
    ``data_parallel``: ranks that draw different sequences (world / sequence-parallel size; default world);
    ``seq_len`` is then the per-rank chunk."""
    dp = data_parallel or world
    if global_batch is not None:
        base = global_batch
    else:
        base = grad_accum * dp  # the sequences per step of (mbs 1, grad_accum)
    cands = [b for b in range(min(max_micro, max(1, base // dp)), 0, -1) if base % (b * dp) == 0]
    modes = [True] if force_checkpointing else ([False, True] if allow_checkpointing else [False])
    tried: List[Dict[str, object]] = []
    for ckpt in modes:
        for b in cands:
            ga = base // (b * dp)
            p = plan_rank(m, world=world, micro_batch=b, seq_len=seq_len, grad_accum=ga,
                          activation_checkpointing=ckpt, **plan_kw)
            tried.append({"micro_batch": b, "checkpointing": ckpt, "total_GiB": round(p.total / GiB, 1)})
            if p.fits(min_headroom):
                return MicroBatchChoice(b, ga, ckpt, p, tried)
    raise ValueError(f"{m.name} at world {world}, seq {seq_len}: no micro-batch fits with "
                     f"{min_headroom:.0%} HBM headroom (even with checkpointing); consider offload_optimizer/param")


def baseline_configs() -> Dict[str, RankPlan]:
    """BASELINE.json configs 2-5 as the MI355X presets run them (launcher.config.presets)."""
    from ..models import get_config

    return {
        "cfg2_llama3_8b_w1": plan_rank(get_config("llama3-8b"), world=1, seq_len=8192, grad_accum=8),
        "cfg3_llama3_8b_w8": plan_rank(get_config("llama3-8b"), world=8, seq_len=8192, grad_accum=8),
        "cfg4_llama3_70b_w8": plan_rank(get_config("llama3-70b"), world=8, seq_len=8192, grad_accum=16,
                                        activation_checkpointing=True),
        "cfg5_mixtral_8x7b_ep8_w8": plan_rank(get_config("mixtral-8x7b"), world=8, seq_len=4096, grad_accum=8,
                                              activation_checkpointing=True, ep_size=8),
    }


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    import json

    from ..models import get_config

    ap = argparse.ArgumentParser(description="per-rank HBM plan of a ZeRO job on MI355X")
    ap.add_argument("--model")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--zero", type=int, default=3)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--ga", type=int, default=8)
    ap.add_argument("--ckpt", action="store_true")
    ap.add_argument("--ep", type=int, default=1)
    ap.add_argument("--auto-mbs", action="store_true", help="size the micro-batch to the plan (keeps mbs x GA)")
    a = ap.parse_args(argv)
    if not a.model:
        print(json.dumps({k: v.summary() for k, v in baseline_configs().items()}, indent=1))
        return 0
    if a.auto_mbs:
        ch = auto_micro_batch(get_config(a.model), world=a.world, seq_len=a.seq, global_batch=a.mbs * a.ga * a.world,
                              zero_stage=a.zero, ep_size=a.ep, force_checkpointing=a.ckpt)
        print(json.dumps(ch.summary(), indent=1))
        return 0
    p = plan_rank(get_config(a.model), world=a.world, zero_stage=a.zero, micro_batch=a.mbs, seq_len=a.seq,
                  grad_accum=a.ga, activation_checkpointing=a.ckpt, ep_size=a.ep)
    print(json.dumps(p.summary(), indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
