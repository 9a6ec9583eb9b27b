"""In-house ZeRO-0/1/2/3 engine over flat per-unit parameter segments (RCCL over xGMI).

This replaces the DeepSpeed engine that the reference shells out to
(``ai_engine/deepspeed_launcher.py:124-238`` emits the config; SURVEY.md §2.5
N1/N4/N5/N6, §2.7 C1-C5, §2.8). It consumes the same knobs (stage, bucket
sizes, gradient clipping, AdamW hyper-parameters, WarmupDecayLR) but is laid
out for MI355X:

Storage (per rank; P = partition world = W for stages 1-3, 1 for stage 0)
    p16_shard   bf16 [sum_g N_g / P]   compute copy of this rank's partition
    master, exp_avg, exp_avg_sq, grad_shard  fp32 [same]  -- ONE buffer each, so
                the optimizer is one fused HIP launch with no host sync
    p16_full    bf16 [sum_g N_g]       stages 1-2 (persistent gathered params)
    grad_full   fp32 [sum_g N_g]       stage 1, and stages 2-3 with local_grad_accum (local
                                       accumulation until the boundary)

Buckets = units: every transformer block is one flat segment (Llama-3-8B:
218 M params, 436 MB bf16; 70B: 856 M, 1.7 GB). That is the MI355X bucket policy
of SURVEY.md §5.8: with 288 GB per GPU we move whole blocks in single, large
RCCL collectives instead of DeepSpeed's 5e8-element buckets.

Schedule (one micro-batch)
    forward : for each unit  -> wait gather(unit) [stage 3], prefetch gather(next),
              unit.forward, free gathered params (the head's are kept for backward)
    backward: for each unit in reverse -> wait gather, prefetch gather(prev),
              unit.backward either accumulates fp32 grads straight into the
              gradient partition (P == 1, ZeRO-0/1: "direct", GEMM beta = 1) or
              writes bf16 grads into a flat scratch segment that is async
              reduce-scattered(avg) (ZeRO-2/3, P > 1) with the fp32 accumulation
              deferred by one unit so RCCL overlaps the next unit's backward.
              With ``local_grad_accum`` (ZeRO-2/3, grad_accum > 1, default "hbm": when
              a full fp32 gradient fits in 15 % of HBM -- Llama-3-8B: 32 GB of 288)
              every micro-batch accumulates fp32 grads directly (like ZeRO-1) and
              each unit is reduce-scattered ONCE per optimizer step, in comm_dtype,
              overlapped with the last micro-batch's backward: 1/GA of DeepSpeed's
              per-micro-batch gradient traffic (FSDP ``no_sync`` pattern); params
              and optimizer state stay partitioned
    step    : grad_stats (sum g^2, #non-finite) -> all_reduce(2 floats) ->
              fused AdamW reading clip coef / overflow flag on device ->
              (stage 1/2) all-gather updated bf16 params. ZeRO-3 on the device runs the
              AdamW as one launch per unit on a side stream (``optimizer_overlap``); the
              next step's forward waits for each unit's update where it first uses it
              (the gather of a partitioned unit, the fetch of an unpartitioned one).
    side streams: the per-step W^T cache rebuild (read only by the backward's dX GEMMs)
              and the MoE dW operand re-layout run beside the compute stream; every
              consumer waits for their events (tests spin those streams to prove it).
"""
from __future__ import annotations

import collections
import contextlib
import math
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from ..models import ModelConfig, StepContext, build_model
from ..models.common import ParamSpec, init_param
from .comm import Comm, DONE, Handle
from .residency import ResidencyPlan, resolve_limit
from ..utils.streams import owned_stream

ALIGN = 64  # elements; keeps every param / shard view 128-byte aligned (bf16) for the HIP kernels


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class EngineConfig:
    zero_stage: int = 3
    micro_batch_size: int = 1
    seq_len: int = 2048
    grad_accum: int = 1
    lr: float = 3e-5
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.01
    grad_clip: float = 1.0
    scheduler: str = "WarmupDecayLR"
    warmup_steps: int = 100
    total_steps: int = 10000
    warmup_min_lr: float = 0.0
    warmup_type: str = "log"  # DeepSpeed WarmupLR default
    comm_dtype: torch.dtype = torch.bfloat16
    # dtype of the ONCE-per-step reduce-scatter of the fp32 local gradient accumulator (local_grad_accum): fp32 by
    # default -- RCCL's ring and the xGMI mesh then reduce the same fp32 values (no bf16 rounding before the sum,
    # equal up to the order of the fp32 additions), for 2x the bytes of one reduce-scatter per step, overlapped with
    # the last backward. comm_dtype (DeepSpeed communication_data_type) keeps governing the
    # per-micro-batch reduce-scatters of the scratch path.
    step_comm_dtype: torch.dtype = torch.float32
    activation_checkpointing: bool = False
    cpu_checkpointing: bool = False
    prefetch: bool = True
    # ZeRO-3 gathered-parameter residency, DeepSpeed semantics (reference config keys
    # stage3_max_live_parameters / stage3_max_reuse_distance / stage3_prefetch_bucket_size,
    # ai_engine/deepspeed_launcher.py:188-190): a gathered unit stays resident after a visit when the
    # parameters fetched before its next visit are <= max_reuse_distance and the resident set stays
    # <= max_live_parameters. "hbm" sizes both to this GPU (live_hbm_fraction of its HBM), so on a
    # 288 GB MI355X a whole Llama-3-8B stays gathered across the micro-batches of a step: one
    # all-gather per unit per optimizer step instead of two per micro-batch. Persistent state
    # (bf16 params, fp32 master/m/v, fp32 grads) stays partitioned 1/W either way.
    max_live_parameters: Any = 1e9
    max_reuse_distance: Any = 1e9
    prefetch_bucket_size: float = 5e8
    # host run-ahead bound for ZeRO-3 gathers: a new gathered buffer is allocated only once the compute stream has
    # finished with the one released this many releases ago (host wait on its event). Without it the host queues
    # gathers for dozens of layers ahead of the GPU, and the released buffers -- record_stream-ed to the collective's
    # stream, so not reusable until that stream drains -- pile up in the caching allocator: at Llama-3-70B rank scale
    # 283-287 GiB reserved for 187.5 GiB allocated and an OOM-retry (free everything, sync, re-malloc) every step;
    # the first step took 10.7 s instead of 4.3 s (tools/diag/r05/resume_probe.py). 0 = unbounded.
    gather_inflight_limit: int = 4
    live_hbm_fraction: float = 0.12
    # 'hbm' residency / W^T-cache sizing leaves at least this fraction of the device free (planner.zero3_budgets)
    hbm_headroom: float = 0.10
    seed: int = 1234
    expert_parallel_size: int = 1
    # Ulysses sequence parallelism (parallel/sp.py): seq_len is then the LOCAL chunk per rank and a
    # group of sequence_parallel_size consecutive ranks holds one sequence of seq_len * size tokens
    sequence_parallel_size: int = 1
    offload_optimizer: str = "none"  # none | cpu | nvme (ZeRO-Offload parity path: parallel/offload.py)
    # ZeRO-Infinity parameter offload (reference offload_param, deepspeed_launcher.py:40, 205-212; ZeRO-3 only):
    # "cpu": the bf16 parameter partition lives in pinned host memory; each gather stages the shard H2D on a
    # side stream and all-gathers from there. "nvme": the partition is a file under nvme_path, read per gather
    # through the C++ AIO engine into a ring of param_buffer_count pinned slots (offload.NvmeParamStore)
    offload_param: str = "none"
    param_buffer_count: int = 5  # offload_param.buffer_count (DeepSpeed default 5)
    # device-driven xGMI mesh transport (parallel/xgmi_mesh.py): "on" = the dense ZeRO parameter all-gathers
    # (a pull over every peer's link at once, out of the peers' symmetric heaps), the dense gradient
    # reduce-scatters (push into the owners' slots + an fp32 rank-order reduce fused with the accumulate) and, at
    # EP > 1, the expert token exchange (parallel/ep.py MeshExpertDispatcher) -- no host synchronisation, so the
    # multi-rank micro-batch loop can be HIP-graph captured; "off" = RCCL rings (the default until an 8-GPU
    # node has measured both: bench.py's post-timing mesh sweep)
    xgmi_mesh: str = "off"
    mesh_min_bytes: int = 0  # dense collectives below this many bytes stay on RCCL
    mesh_timeout_s: float = 120.0  # a device-side wait past this records an error (XgmiMesh.check) and returns
    # mesh EP receive capacity: None = dropless (every rank's receive slot holds the worst case, W x T x k rows; the
    # expert activations are static worst-case tensors when they fit ep_static_hbm_fraction of HBM -- capturable --
    # else sized per dispatch by one host read); a number = a static capacity of that many times the balanced share,
    # and a routing that overflows it raises at the step boundary (check_transport)
    ep_capacity_factor: Optional[float] = None
    ep_static_hbm_fraction: float = 0.10
    # expert weight gradients: keep each micro-batch's (dY, X) per expert and run one dW GEMM per expert over
    # the concatenated micro-batches at the last one (K = GA x tokens: the fp32 gradient is read and written
    # once per step instead of once per micro-batch). Only with direct fp32 gradient targets; "auto" = on
    # when grad_accum > 1. Stashed operands are capped by defer_wgrad_budget_gb (flushed early above it).
    defer_expert_wgrad: Any = "auto"
    defer_wgrad_budget_gb: float = 48.0
    # the expert groups' gradient statistics (sum of squares, #non-finite) tallied by the grouped dW GEMM's
    # epilogue at the last micro-batch instead of a separate pass over the expert gradients (single rank:
    # the stored gradient is then final); falls back to ops.grad_stats whenever a weight was not covered.
    # A/B on Mixtral 2-layer: 133.2k -> 136.3k tokens/s, identical grad norm (profiles/fused_expert_stats_ab_r03.json)
    fused_expert_grad_stats: bool = True
    # ZeRO-3 on the device (no offload, no mesh): the AdamW of step s runs on a side stream as one launch per
    # parameter group in forward order, and step s+1's forward waits for each group's update where it fetches
    # the group instead of for the whole update -- the bandwidth-bound optimizer overlaps the first layers'
    # compute (element for element the same arithmetic as the single flat launch). Off by default: the round-4
    # closing A/B measured it neutral for Llama-3-8B and Mixtral (profiles/optimizer_overlap_onoff_closing_r04.txt)
    optimizer_overlap: bool = False
    nvme_path: Optional[str] = None
    param_nvme_path: Optional[str] = None  # offload_param.nvme_path (defaults to nvme_path)
    # ZeRO-2/3 gradients: True = accumulate fp32 locally and reduce-scatter once per optimizer step;
    # False = reduce-scatter every micro-batch (DeepSpeed); "hbm" = True when GA > 1 and the full fp32
    # gradient fits in local_grad_hbm_fraction of the device
    local_grad_accum: Any = "hbm"
    local_grad_hbm_fraction: float = 0.15
    offload_buffer_count: int = 4  # NVMe swap ring slots (offload_optimizer.buffer_count)
    aio_threads: int = 8  # C++ AIO engine: I/O threads (DeepSpeed aio thread_count x queue_depth)
    aio_block_size: int = 8 << 20  # bytes per I/O piece (DeepSpeed aio block_size)
    wall_clock_breakdown: bool = False  # per-phase HIP-event timers (utils/timers.py)
    # parameter all-gathers on their own communicator (own RCCL stream), so a prefetch gather of the
    # next block and the reduce-scatter of the previous block's gradients run concurrently on xGMI
    separate_gather_comm: bool = True
    tuned_gemms: bool = True  # load TunableOp results for this model if present (utils/gemm_tuning.py)
    # checkpoints carry the full 16-bit module state dict in mp_rank_00_model_states.pt (DeepSpeed does for
    # stages 0-2; for stage 3 only with stage3_gather_16bit_weights_on_model_save, which the reference sets:
    # deepspeed_launcher.py:74, 192) -- gathered group by group at save time (ckpt/checkpoint.py)
    gather_16bit_weights_on_model_save: bool = True
    # keep W^T of the big 2-D weights while the compute copy is stationary (P == 1, ZeRO-0/1/2): the
    # input-gradient GEMMs then run with both operands K-contiguous (refreshed once per optimizer step)
    transposed_weight_cache: bool = True
    # ZeRO-3 (P > 1): groups the residency plan holds gathered for the whole step get the W^T cache too,
    # while the caches fit in this fraction of HBM (Llama-3-8B: 14 GiB) and in what the HBM plan leaves
    tcache_hbm_fraction: float = 0.08
    # W^T cache also for expert-stacked [E, out, in] weights of never-gathered groups (expert dX GEMMs read
    # K-contiguous weights), within tcache_hbm_fraction of the device
    expert_weight_cache: bool = True
    init_device: str = "auto"  # "cpu" gives bit-identical init on any device (tests); auto: cpu below 1e9 params
    # replay the GA micro-batches of a step (forward + backward + gradient accumulation) as ONE captured
    # HIP graph: one launch instead of ~30 kernel launches per layer per micro-batch, for models whose
    # step is launch-bound (GPT-2-small, small Llama). Needs a step with no collective and no host sync
    # inside the micro-batch loop (single rank, dense model, no offload, bf16); otherwise eager.
    hip_graphs: bool = False
    # once a step has non-finite gradients every later update is skipped on the device too (halt-on-NaN
    # jobs whose host runs a step ahead: the state at exit is the state before the poisoned step)
    nan_latch: bool = False
    # DeepSpeed prescale_gradients / gradient_predivide_factor (reference deepspeed_launcher.py:61-62, 168-169):
    # prescale: every gradient contribution is pre-divided by the factor (folded into the loss-gradient scale),
    # reduced with SUM and post-multiplied by factor / world (folded into the accumulate alpha); otherwise
    # reductions average (AVG)
    prescale_gradients: bool = False
    gradient_predivide_factor: float = 1.0
    # stage3_param_persistence_threshold (reference :73, :191): under ZeRO-3 with W > 1, parameters with fewer
    # elements stay replicated on every rank (their own P == 1 group per unit: never gathered, gradients
    # all-reduced); 0 disables
    param_persistence_threshold: float = 0.0
    fp16: bool = False  # dynamic loss scaling path (reference fp16 block)
    loss_scale: float = 0.0  # 0 = dynamic
    initial_scale_power: int = 16
    loss_scale_window: int = 1000
    hysteresis: int = 2
    min_loss_scale: float = 1.0

    @property
    def tokens_per_micro(self) -> int:
        return self.micro_batch_size * self.seq_len


class FlatGroup:
    """One parameter group (= one unit) as a flat, ALIGN-padded, W-divisible segment."""

    def __init__(self, idx: int, name: str, specs: List[ParamSpec], part_world: int, kind: str = "dense",
                 comm: Optional[Comm] = None):
        self.idx, self.name, self.specs = idx, name, specs
        self.prefix = name[:-len(".persist")] if name.endswith(".persist") else name  # parameter-name prefix
        self.kind, self.P, self.comm = kind, part_world, comm
        self.layout: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
        off = 0
        for s in specs:
            self.layout[s.name] = (off, tuple(s.shape))
            off += _round_up(s.numel, ALIGN)
        self.numel = _round_up(max(off, 1), ALIGN * part_world)
        self.shard_numel = self.numel // part_world
        self.gcomm = comm  # communicator for parameter all-gathers (the engine may give it its own)
        self.real_numel = sum(s.numel for s in specs)
        self.shard_off = 0
        self.full_off = 0

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for s in self.specs:
            off, shape = self.layout[s.name]
            out[s.name] = flat.narrow(0, off, s.numel).view(shape)
        return out


class _Scaled:
    """Pending-reduction payload: multiply `t` by `factor` once the collective completed (prescale post-scale);
    `keep` holds the collective's input alive until then."""

    def __init__(self, t: torch.Tensor, factor: float, keep: Any = None):
        self.t, self.factor, self.keep = t, factor, keep


class _MeshRS:
    """Pending mesh reduce-scatter of a pooled bf16 gradient buffer (already accumulated into the shard by the
    reduce kernel): the buffer returns to the pool once the collective completed."""

    def __init__(self, src: torch.Tensor):
        self.src = src


class LossScaler:
    """fp16 dynamic loss scaler whose state lives on the device (DeepSpeed fp16 block semantics, reference
    deepspeed_launcher.py:175-183).

    ``state`` = [scale, 1/scale, good steps, hysteresis left] (fp32). The cross-entropy kernel multiplies
    the loss gradient by ``state[0]``, AdamW unscales with ``state[1]`` and a one-thread kernel applies the
    update rule from the step's non-finite count: a step never reads the scale on the host, so the
    trainer's one-step-behind run-ahead holds on the fp16 path too. ``scale`` (a host read) is for
    checkpoints, logs and tests.
    """

    def __init__(self, cfg: EngineConfig, device):
        self.dynamic = cfg.loss_scale == 0
        s0 = float(cfg.loss_scale if cfg.loss_scale else 2.0 ** cfg.initial_scale_power)
        self.window, self.hyst, self.min_scale = cfg.loss_scale_window, cfg.hysteresis, cfg.min_loss_scale
        self.state = torch.tensor([s0, 1.0 / s0, 0.0, float(cfg.hysteresis)], dtype=torch.float32, device=device)

    @property
    def scale(self) -> float:
        return float(self.state[0])

    def update_(self, stats: torch.Tensor) -> None:
        """Apply the DeepSpeed rule to the step whose non-finite count is ``stats[1]`` (device, no sync)."""
        if self.dynamic:
            ops.loss_scale_update_(self.state, stats, self.window, self.hyst, self.min_scale)

    def state_dict(self) -> Dict[str, Any]:
        scale, _, good, hyst = (float(x) for x in self.state.tolist())
        return {"cur_scale": scale, "cur_iter_good": int(good), "cur_hysteresis": int(hyst),
                "dynamic": self.dynamic}

    def load_state_dict(self, d: Dict[str, Any]) -> None:
        scale = float(d["cur_scale"])
        good = float(d.get("cur_iter_good", 0))
        hyst = float(d.get("cur_hysteresis", self.hyst))
        self.state.copy_(torch.tensor([scale, 1.0 / scale, good, hyst], dtype=torch.float32))


def lr_at(cfg: EngineConfig, step: int) -> float:
    """LR for optimizer step `step` (1-based), DeepSpeed WarmupLR / WarmupDecayLR / WarmupCosineLR."""
    it = step - 1
    lo, hi, wu = cfg.warmup_min_lr, cfg.lr, max(1, cfg.warmup_steps)
    if cfg.scheduler in ("constant", "none", None):
        return hi
    if it < wu:
        if cfg.warmup_type == "log":
            gamma = math.log(it + 1) / math.log(wu)
        else:
            gamma = it / wu
        return lo + (hi - lo) * gamma
    if cfg.scheduler == "WarmupLR":
        return hi
    total = max(cfg.total_steps, wu + 1)
    frac = max(0.0, (total - it) / max(1, total - wu))
    if cfg.scheduler == "WarmupCosineLR":
        return hi * 0.5 * (1 + math.cos(math.pi * (1 - frac)))
    return hi * frac  # WarmupDecayLR: linear decay to 0 at total_num_steps


def _state_tensor(name: str) -> property:
    """An engine state tensor (fp32 master / moments / gradient partition, compute copy) read from outside the
    step: waits for an overlapped optimizer update still writing it (cfg.optimizer_overlap). The fetch path reads
    the raw tensor after waiting for its own group only."""
    key = "_st_" + name

    def get(self):
        if self.__dict__.get("_opt_pending"):
            self.join_optimizer()
        return self.__dict__[key]

    def put(self, v) -> None:
        self.__dict__[key] = v
    return property(get, put)


class ZeroEngine:
    master = _state_tensor("master")
    exp_avg = _state_tensor("exp_avg")
    exp_avg_sq = _state_tensor("exp_avg_sq")
    grad_shard = _state_tensor("grad_shard")
    p16_shard = _state_tensor("p16_shard")

    def __init__(self, model_cfg: ModelConfig, cfg: EngineConfig, device: torch.device, comm: Optional[Comm] = None,
                 ep_comm: Optional[Comm] = None):
        self._opt_pending: Dict[int, Any] = {}  # group -> event of its overlapped update (cfg.optimizer_overlap)
        self._opt_stream = None
        # the stream the engine computes on (captured at construction): join_optimizer orders IT after the overlapped
        # updates, whatever stream happens to be current where the join is called from
        self._compute_stream = torch.cuda.current_stream(device) if device.type == "cuda" else None
        self._opt_delay_cycles = 0  # test hook: spin the optimizer stream first (a missing wait then reads stale state)
        self.mcfg, self.cfg, self.device = model_cfg, cfg, device
        self.comm = comm or Comm()
        self.W, self.rank = self.comm.world, self.comm.rank
        self.stage = cfg.zero_stage
        assert self.stage in (0, 1, 2, 3), "ZeRO stage must be 0..3"
        self.P = 1 if self.stage == 0 else self.W
        # expert parallelism: experts live on EP ranks, sharded (ZeRO) only over expert-data-parallel ranks
        self.ep_size = max(1, cfg.expert_parallel_size) if model_cfg.n_experts else 1
        if self.ep_size > 1 and self.W > 1:
            from .ep import build_ep_comms
            self.ep_comm, self.edp_comm = build_ep_comms(self.ep_size, self.comm)
        else:
            self.ep_size = 1
            self.ep_comm, self.edp_comm = None, self.comm
        ep_comm = ep_comm or self.ep_comm
        self.ep_comm = ep_comm
        self.sp_size, self.sp_comm = max(1, cfg.sequence_parallel_size), None
        if self.sp_size > 1 and self.W > 1:
            from .sp import build_sp_comm
            self.sp_comm = build_sp_comm(self.sp_size, self.comm)
        else:
            self.sp_size = 1
        ep_rank = self.ep_comm.rank if self.ep_comm is not None else 0
        self.gather_comm = self.comm
        if cfg.separate_gather_comm and self.W > 1 and self.stage > 0:
            self.gather_comm = self.comm.duplicate()
        groups, stages = build_model(model_cfg, ep_rank, self.ep_size)
        groups, stages, self._orig_groups = self._split_persistent(groups, stages)
        self.stages = [(u, tuple(gi) if isinstance(gi, (tuple, list)) else (gi,)) for u, gi in stages]
        self.groups = []
        for i, grp in enumerate(groups):
            name, specs = grp[0], grp[1]
            kind = grp[2] if len(grp) > 2 else "dense"
            if kind == "expert":
                comm_g = self.edp_comm if self.edp_comm is not None else Comm()
                P_g = 1 if self.stage == 0 else comm_g.world
            elif kind == "persist":
                comm_g, P_g = self.comm, 1  # replicated on every rank, gradients all-reduced
            else:
                comm_g, P_g = self.comm, self.P
            fg = FlatGroup(i, name, specs, P_g, kind, comm_g)
            fg.gcomm = self.gather_comm if kind != "expert" else comm_g
            self.groups.append(fg)
        self.has_experts = any(g.kind == "expert" for g in self.groups)
        # fused expert gradient statistics: only where the gradient the dW epilogue stores is the final one
        # (no reduction, no EP rescale, no post-scale after it)
        self._xstats_weights = sum(len(g.specs) for g in self.groups if g.kind == "expert")
        self._xstats = None
        self._xstats_ok = False
        if (self.has_experts and cfg.fused_expert_grad_stats and self.W == 1 and self.ep_size == 1
                and (self.ep_comm is None or self.ep_comm.world == 1) and not cfg.prescale_gradients):
            self._xstats = torch.zeros(2, dtype=torch.float32, device=self.device)
        soff = foff = 0
        for g in self.groups:
            g.shard_off, g.full_off = soff, foff
            soff += g.shard_numel
            foff += g.numel
        self.shard_total, self.full_total = soff, foff
        # local fp32 gradients exist only for groups that are reduce-scattered (P > 1); a P == 1 group
        # (e.g. experts at EP == W) accumulates straight into its fp32 shard
        goff = 0
        for g in self.groups:
            g.gfull_off = goff
            goff += g.numel if g.P > 1 else 0
        self.gfull_total = goff
        self.mesh = None
        self.ep_mesh = None
        self._transport_word = None
        self._init_mesh(model_cfg)
        # compute dtype: bf16, or fp16 for the DeepSpeed "fp16" block -- every HIP kernel has an f16
        # instantiation (f16 MFMA in attention) and the dynamic loss scaler guards the fp16 range
        self.dtype = torch.float16 if cfg.fp16 else torch.bfloat16
        self.is_cuda = device.type == "cuda"
        self.tuned_gemm_files: List[str] = []
        if self.is_cuda and cfg.tuned_gemms:
            from ..utils.gemm_tuning import enable_tuned_gemms
            self.tuned_gemm_files = enable_tuned_gemms(model_cfg.name)
        self._alloc()
        self._init_params()
        self._pver = 0  # bumped whenever the bf16 compute copy changes
        self._tcache: Dict[int, Tuple[int, Dict[str, torch.Tensor]]] = {}
        self._tcache_ev: Dict[int, Any] = {}  # group -> event of a side-stream cache rebuild not yet waited for
        self._tnames: Dict[int, List[Tuple[str, Tuple[int, ...]]]] = {}
        self._expert_wt = cfg.expert_weight_cache
        if cfg.transposed_weight_cache:
            # 2-D weights always; expert-stacked [E, out, in] weights within tcache_hbm_fraction of the device
            budget = (cfg.tcache_hbm_fraction * torch.cuda.get_device_properties(device).total_memory
                      if device.type == "cuda" else math.inf)
            used = 0
            for g in self.groups:
                if self.stage < 3 or g.P == 1:
                    names = [(sp.name, tuple(sp.shape)) for sp in g.specs if sp.tcache and len(sp.shape) == 2]
                    stacked = [(sp.name, tuple(sp.shape)) for sp in g.specs
                               if sp.tcache and len(sp.shape) == 3 and self._expert_wt]
                    nbytes = sum(math.prod(shp) for _, shp in stacked) * 2
                    if stacked and used + nbytes <= budget:
                        names += stacked
                        used += nbytes
                    if names:
                        self._tnames[g.idx] = names
        self.step_count = 0
        self.scaler = LossScaler(cfg, device) if cfg.fp16 else None
        # [sum g^2, #non-finite, host flags]: the flags slot rides the stats all-reduce, so ranks agree on
        # host-side events (preemption) without a collective or a host read of their own
        self.stats = torch.zeros(3, dtype=torch.float32, device=device)
        self.host_flag = 0.0  # set by the trainer before a step (e.g. 1.0 = preemption notice on this rank)
        self.sync_flags = False  # all-reduce the flag even when nothing else needs a collective (P == 1, W > 1)
        self._nan_latch = torch.zeros(1, dtype=torch.float32, device=device) if cfg.nan_latch else None
        self.loss_acc = torch.zeros((), dtype=torch.float32, device=device)
        from ..ops.rope import rope_tables
        if model_cfg.arch in ("llama", "mixtral"):
            S = max(cfg.seq_len, 1)
            cos, sin = rope_tables(model_cfg.head_dim, S * self.sp_size, model_cfg.rope_theta, device,
                                   model_cfg.rope_scaling)
            off = (self.sp_comm.rank if self.sp_comm is not None else 0) * S  # this rank's chunk: global positions
            self.rope = (cos[off:off + S].contiguous(), sin[off:off + S].contiguous())
        else:
            self.rope = None
        # group visit bookkeeping (tied weights appear twice)
        self._bwd_last_visit: Dict[int, int] = {}
        for si, (_, gis) in enumerate(self.stages):
            for gi in gis:
                self._bwd_last_visit[gi] = min(si, self._bwd_last_visit.get(gi, si))
        self._live: Dict[int, Tuple[torch.Tensor, Handle]] = {}
        self._free_events: "collections.deque" = collections.deque()  # gathered-buffer releases (run-ahead bound)
        first_use: List[int] = []
        for _, gis in self.stages:
            first_use += [gi for gi in gis if gi not in first_use]
        self._opt_order = first_use + [g.idx for g in self.groups if g.idx not in first_use]
        self._build_live_plan()
        if cfg.transposed_weight_cache and self.stage == 3:
            self._add_resident_tcache()
        self._gbuf_pool: Dict[int, List[torch.Tensor]] = {}
        self._act_offload = None
        self.fault_inject_nan = False  # fault injection: poison one gradient element on the next micro-step
        self._graph: Optional[Dict[str, Any]] = None  # captured micro-batch loop (cfg.hip_graphs)
        self._graph_state = "cold"  # cold -> warm (one eager step done) | failed (capture refused)
        from ..utils.timers import PhaseTimers
        self.timers = PhaseTimers(device, enabled=cfg.wall_clock_breakdown)
        self.hooks: List[Any] = []  # callables(engine, metrics) after each step (NaN trap, monitors)
        self.pre_step_hooks: List[Any] = []  # callables(engine) before the optimizer touches master/m/v

    def _init_mesh(self, model_cfg: ModelConfig) -> None:
        """Build the xGMI mesh heaps (cfg.xgmi_mesh == "on"): the world heap holds this rank's bf16 parameter
        partition (peers pull their gathers from it) and the reduce-scatter slots; the EP heap the token slots."""
        c = self.cfg
        if c.xgmi_mesh not in ("on", "off"):
            raise ValueError(f"xgmi_mesh must be 'on' or 'off', got {c.xgmi_mesh!r}")
        if c.xgmi_mesh != "on" or not self.is_cuda_dev() or self.W == 1:
            return
        if self.comm.backend not in ("nccl", "gloo", "shadow") or c.offload_optimizer != "none" or \
                c.offload_param != "none":
            return  # host-resident partitions keep the RCCL path
        from .xgmi_mesh import XgmiMesh, rs_region_bytes
        dense = [g for g in self.groups if self._mesh_group(g)]
        regions = {"p16": (self.shard_total * 2, 1)}
        if dense and self.stage in (2, 3):
            # fp32 slots when the once-per-step reduce of the local accumulator travels in fp32
            esz = 4 if (self._want_local_grads() and c.step_comm_dtype == torch.float32) else 2
            regions["rs"] = (rs_region_bytes(self.W, max(g.shard_numel for g in dense), esz), 2)
        self.mesh = XgmiMesh(self.comm, self.device, regions, c.mesh_timeout_s)
        if self.ep_size > 1 and self.ep_comm is not None and self.ep_comm.world > 1:
            from .ep import MeshExpertDispatcher
            dt = torch.float16 if c.fp16 else torch.bfloat16
            from .ep import static_dispatch_fits
            rows = c.tokens_per_micro * model_cfg.top_k
            sized = False
            if c.ep_capacity_factor is None:
                hbm = torch.cuda.get_device_properties(self.device).total_memory
                sized = not static_dispatch_fits(rows * self.ep_comm.world, model_cfg.d_model, model_cfg.ffn_dim,
                                                 model_cfg.n_layers, c.activation_checkpointing, hbm,
                                                 c.ep_static_hbm_fraction)
            self.ep_mesh = MeshExpertDispatcher(self.ep_comm, model_cfg.n_experts, self.device, rows,
                                                model_cfg.d_model, dt, c.ep_capacity_factor,
                                                timeout_s=c.mesh_timeout_s, sized_output=sized)

    def is_cuda_dev(self) -> bool:
        return self.device.type == "cuda"

    def _mesh_group(self, g: "FlatGroup") -> bool:
        """Dense group partitioned over the whole world: its gathers / reductions can ride the world mesh."""
        return g.kind != "expert" and g.P == self.W and g.P > 1 and g.comm is self.comm

    def _mesh_ok(self, g: "FlatGroup", t: torch.Tensor) -> bool:
        return (self.mesh is not None and self._mesh_group(g)
                and t.numel() * t.element_size() >= self.cfg.mesh_min_bytes)

    def check_transport(self) -> None:
        """Raise if a mesh wait timed out or an EP dispatch overflowed its receive capacity (host reads of two device
        words: the trainer calls this at every step boundary where it already syncs, and train_step after the
        optimizer when ``check_transport_every`` says so). A timed-out wait makes every later mesh kernel return at
        once (the sticky error word), so the step that raised trained on nothing it could not trust: the caller
        halts the job and the supervisor resumes from the last verified checkpoint."""
        for m in (self.mesh, self.ep_mesh.mesh if self.ep_mesh is not None else None):
            if m is not None:
                m.check()
        if self.ep_mesh is not None and self.ep_mesh.overflowed():
            what = ("internal error: the dropless receive slot overflowed" if self.ep_mesh.dropless else
                    f"a routing overflowed the mesh EP receive capacity ({self.ep_mesh.C} rows, ep_capacity_factor "
                    f"{self.cfg.ep_capacity_factor}); set ep_capacity_factor to None (dropless)")
            raise RuntimeError(f"xGMI mesh: {what}")

    def transport_word(self) -> torch.Tensor:
        """fp32 [1] on the device: 1 if a mesh wait timed out, + 2 if an EP dispatch overflowed its receive
        capacity; 0 without a mesh. The trainer reads it one step late with the NaN-trap report (no sync)."""
        if self._transport_word is None:
            self._transport_word = torch.zeros(1, dtype=torch.float32, device=self.device)
        meshes = [m for m in (self.mesh, self.ep_mesh.mesh if self.ep_mesh is not None else None) if m is not None]
        if not meshes:
            return self._transport_word
        from .xgmi_mesh import ST_ERR, ST_OVF
        w = self._transport_word
        w.zero_()
        for m in meshes:
            w += (m.state[ST_ERR] != 0).float() + 2.0 * (m.state[ST_OVF] != 0).float()
        return w.clamp_(max=3.0)

    def _split_persistent(self, groups, stages):
        """stage3_param_persistence_threshold: move each unit's small tensors (norm weights, biases) into a
        replicated "<unit>.persist" group beside the partitioned one. Returns (groups, stages, originals);
        originals = [(original index, name, specs, new group indices)] keeps initialisation identical to the
        unsplit layout."""
        thr = self.cfg.param_persistence_threshold
        orig = []
        if not (thr > 0 and self.stage == 3 and self.W > 1):
            for i, grp in enumerate(groups):
                orig.append((i, grp[0], grp[1], (i,)))
            return groups, stages, orig
        out, remap = [], {}
        for i, grp in enumerate(groups):
            name, specs = grp[0], grp[1]
            kind = grp[2] if len(grp) > 2 else "dense"
            small = [sp for sp in specs if sp.numel < thr] if kind == "dense" else []
            big = [sp for sp in specs if sp not in small]
            idx = []
            if big:
                idx.append(len(out))
                out.append((name, big, kind))
            if small:
                idx.append(len(out))
                out.append((name + ".persist" if big else name, small, "persist"))
            remap[i] = tuple(idx)
            orig.append((i, name, specs, tuple(idx)))
        new_stages = []
        for u, gi in stages:
            gis = tuple(gi) if isinstance(gi, (tuple, list)) else (gi,)
            new_stages.append((u, tuple(j for g in gis for j in remap[g])))
        return out, new_stages, orig

    # ------------------------------------------------------------------ storage
    def _alloc(self) -> None:
        dev, n = self.device, self.shard_total
        f32 = dict(dtype=torch.float32, device=dev)
        self.offload = None
        if self.cfg.offload_optimizer in ("cpu", "nvme"):
            from .offload import HostOffloadOptimizer
            self.offload = HostOffloadOptimizer(n, dev, self.cfg.offload_optimizer, self.cfg.nvme_path, self.rank,
                                                buffer_count=self.cfg.offload_buffer_count,
                                                aio_threads=self.cfg.aio_threads,
                                                aio_block_size=self.cfg.aio_block_size,
                                                dtype=torch.float16 if self.cfg.fp16 else torch.bfloat16)
            self.master, self.exp_avg, self.exp_avg_sq = (self.offload.master, self.offload.exp_avg,
                                                          self.offload.exp_avg_sq)
        else:
            self.master = torch.zeros(n, **f32)
            self.exp_avg = torch.zeros(n, **f32)
            self.exp_avg_sq = torch.zeros(n, **f32)
        self.grad_shard = torch.zeros(n, **f32)
        self.param_host = self.cfg.offload_param in ("cpu", "nvme") and self.stage == 3
        self.param_nvme = None
        if self.param_host and self.cfg.offload_param == "nvme":
            from .offload import NvmeParamStore
            self.param_nvme = NvmeParamStore(n, self.dtype, self.cfg.param_nvme_path or self.cfg.nvme_path, self.rank,
                                             max(g.shard_numel for g in self.groups),
                                             buffer_count=self.cfg.param_buffer_count, cuda=self.is_cuda,
                                             aio_threads=self.cfg.aio_threads,
                                             aio_block_size=self.cfg.aio_block_size)
            self.p16_shard = self.param_nvme.mapped  # cold paths (checkpoints, host optimizer) use the mapping
            self._h2d = owned_stream(dev, "param-h2d", owner=self) if self.is_cuda else None
            self._p16_ready = None
        elif self.param_host:
            self.p16_shard = torch.zeros(n, dtype=self.dtype, pin_memory=self.is_cuda)
            self._h2d = owned_stream(dev, "param-h2d", owner=self) if self.is_cuda else None
            self._p16_ready = None  # event: host bf16 partition final (after the device AdamW's D2H)
        elif self.mesh is not None:  # peers pull their gathers straight out of this rank's heap
            self.p16_shard = self.mesh.region_tensor("p16", self.dtype, n)
        else:
            self.p16_shard = torch.zeros(n, dtype=self.dtype, device=dev)
        self.p16_full = None
        self.grad_full = None
        if self.stage == 0:
            self.p16_full = self.p16_shard  # P == 1: shard == full
        elif self.stage in (1, 2):
            self.p16_full = torch.zeros(self.full_total, dtype=self.dtype, device=dev)
        self.local_grads = self._want_local_grads()
        if self.stage == 1 or self.local_grads:
            self.grad_full = torch.zeros(self.gfull_total, **f32)

    def _want_local_grads(self) -> bool:
        """ZeRO-2/3: accumulate fp32 gradients locally across micro-batches (one reduce-scatter per step)?"""
        v = self.cfg.local_grad_accum
        if self.stage not in (2, 3) or not any(g.P > 1 for g in self.groups):
            return False
        if isinstance(v, str):
            if v not in ("hbm", "auto"):
                raise ValueError(f"local_grad_accum must be a bool or 'hbm', got {v!r}")
            if self.cfg.grad_accum <= 1 or self.device.type != "cuda":
                return False
            hbm = torch.cuda.get_device_properties(self.device).total_memory
            return self.gfull_total * 4 <= self.cfg.local_grad_hbm_fraction * hbm
        return bool(v)

    def _init_params(self) -> None:
        init_dev = self.cfg.init_device
        if init_dev == "auto":
            init_dev = "cpu" if sum(g.real_numel for g in self.groups) < 1e9 else self.device.type
        gen = torch.Generator(device=init_dev)
        for oi, oname, ospecs, new_idx in self._orig_groups:
            # initialise the ORIGINAL unit layout (seeded by its index), so a persistence split does not change
            # any value; then scatter its tensors into the group(s) that hold them now
            og = FlatGroup(oi, oname, ospecs, 1)
            full = torch.zeros(og.numel, dtype=torch.float32, device=init_dev)
            views = og.views(full)
            gseed = self.cfg.seed * 1000003 + oi
            gen.manual_seed(gseed)
            for s in ospecs:
                init_param(s, views[s.name], gen, gseed)
            for gi in new_idx:
                g = self.groups[gi]
                if len(new_idx) == 1 and g.numel == og.numel:
                    gfull = full.to(self.device)
                else:
                    gfull = torch.zeros(g.numel, dtype=torch.float32, device=init_dev)
                    gv = g.views(gfull)
                    for s in g.specs:
                        gv[s.name].copy_(views[s.name])
                    gfull = gfull.to(self.device)
                r0 = (g.comm.rank if g.P > 1 else 0) * g.shard_numel
                self.master.narrow(0, g.shard_off, g.shard_numel).copy_(gfull.narrow(0, r0, g.shard_numel))
                if self.p16_full is not None and self.p16_full is not self.p16_shard:
                    self.p16_full.narrow(0, g.full_off, g.numel).copy_(gfull)
                del gfull
            del full
        self._p16_from_master()

    def _p16_from_master(self) -> None:
        self.join_optimizer()
        self._pver = getattr(self, "_pver", 0) + 1
        if self.offload is not None:
            self.offload.push_params(self.p16_shard)
        elif self.param_host:
            self._p16_to_host()
        else:
            self._mesh_quiesce()
            ops.cast_f32_bf16_(self.p16_shard, self.master)  # bf16 or fp16 compute copy
            self._mesh_publish()

    def _mesh_quiesce(self) -> None:
        """Mesh: before this rank overwrites its parameter partition, every rank finished its reads of it."""
        if self.mesh is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self.mesh.stream("ag"))
            self.mesh.quiesce()

    def _mesh_publish(self) -> None:
        if self.mesh is not None:
            self.mesh.publish()

    def _p16_to_host(self) -> None:
        """offload_param with the optimizer on the device: bf16(master) chunk by chunk into a device scratch,
        then D2H into the pinned host partition (stream-ordered, no host sync)."""
        n, step = self.shard_total, 1 << 26
        if self.param_nvme is not None:
            # NVMe: cast a slot's worth on the device, D2H into the pinned slot, write it to the file
            scratch = torch.empty(min(n, self.param_nvme.slot_elems), dtype=self.dtype, device=self.device)

            def produce(off: int, ln: int, slot: torch.Tensor) -> None:
                if self.is_cuda:
                    ops.cast_f32_bf16_(scratch[:ln], self.master.narrow(0, off, ln))
                    slot.copy_(scratch[:ln], non_blocking=True)
                    torch.cuda.current_stream(self.device).synchronize()  # the file write reads the slot
                else:
                    slot.copy_(self.master.narrow(0, off, ln))
            self.param_nvme.write(produce)
            return
        scratch = torch.empty(min(n, step), dtype=self.dtype, device=self.device)
        for off in range(0, n, step):
            ln = min(step, n - off)
            if self.is_cuda:
                ops.cast_f32_bf16_(scratch[:ln], self.master.narrow(0, off, ln))
            else:
                scratch[:ln].copy_(self.master.narrow(0, off, ln))
            self.p16_shard.narrow(0, off, ln).copy_(scratch[:ln], non_blocking=True)
        if self.is_cuda:
            self._p16_ready = torch.cuda.Event()
            self._p16_ready.record()

    def _gather_from_host(self, g: FlatGroup) -> Tuple[torch.Tensor, Handle]:
        """offload_param: stage the host shard H2D on the side stream and all-gather from there (the RCCL work
        is ordered after the copy, not after the compute queued so far). NVMe: the shard is first read from the
        file into a pinned ring slot (C++ AIO), which is released once its H2D copy has run."""
        slot = None
        if self.param_nvme is not None:
            slot, host = self.param_nvme.read(g.shard_off, g.shard_numel)
        else:
            host = self._shard16(g)
        if not self.is_cuda:
            stage = host.clone()
            if g.P == 1:
                return stage, DONE
            buf = torch.empty(g.numel, dtype=self.dtype, device=self.device)
            return buf, g.gcomm.all_gather(buf, stage, async_op=True)
        with torch.cuda.stream(self._h2d):
            if self._p16_ready is not None:
                self._h2d.wait_event(self._p16_ready)
            stage = torch.empty(g.shard_numel, dtype=self.dtype, device=self.device)
            stage.copy_(host, non_blocking=True)
            if slot is not None:
                done = torch.cuda.Event()
                done.record(self._h2d)
                self.param_nvme.release_after(slot, done)
            if g.P == 1:
                ev = torch.cuda.Event()
                ev.record(self._h2d)
                return stage, Handle(post=lambda: torch.cuda.current_stream(self.device).wait_event(ev))
            buf = torch.empty(g.numel, dtype=self.dtype, device=self.device)
            h = g.gcomm.all_gather(buf, stage, async_op=True)
            # the gather was issued on the H2D stream: the consumer waits for the collective (RCCL work) AND for the
            # H2D stream itself -- a communicator that runs the gather inline on the issuing stream (a synchronous
            # shadow rank) returns a done handle, and the compute stream would read buf unordered (stream audit)
            ev = torch.cuda.Event()
            ev.record(self._h2d)
            return buf, Handle(post=lambda: (h.wait(), torch.cuda.current_stream(self.device).wait_event(ev)))

    # ------------------------------------------------------------------ params
    def _all_gather(self, g: FlatGroup, out: torch.Tensor, shard: torch.Tensor) -> Handle:
        if self._mesh_ok(g, out):
            m = self.mesh
            return m.run_async(lambda: m.all_gather_pull(out, shard), [out])
        return g.gcomm.all_gather(out, shard, async_op=True)

    def _shard16(self, g: FlatGroup) -> torch.Tensor:
        return self._st_p16_shard.narrow(0, g.shard_off, g.shard_numel)  # (no join: _issue_gather waited)

    def _issue_gather(self, gi: int) -> None:
        if gi in self._live:
            return
        if self.groups[gi].P > 1:  # the gather reads the shard: the group's overlapped update lands first
            self._wait_update(gi)
        g = self.groups[gi]
        if self.stage < 3:
            flat = self.p16_full.narrow(0, g.full_off, g.numel)
            self._live[gi] = (flat, DONE)
        elif self.param_host:
            self._live[gi] = self._gather_from_host(g)
        elif g.P == 1:
            self._live[gi] = (self._shard16(g), DONE)
        else:
            self._bound_run_ahead()
            buf = torch.empty(g.numel, dtype=self.dtype, device=self.device)
            self._live[gi] = (buf, self._all_gather(g, buf, self._shard16(g)))

    def _bound_run_ahead(self) -> None:
        """Host-wait until the compute stream is done with the gathered buffer released gather_inflight_limit
        releases ago (cfg.gather_inflight_limit; PyTorch FSDP's all-gather rate limiter works the same way)."""
        lim = self.cfg.gather_inflight_limit
        if lim <= 0 or not self.is_cuda or torch.cuda.is_current_stream_capturing():
            return
        while len(self._free_events) >= lim:
            self._free_events.popleft().synchronize()

    def _released(self, gi: int) -> None:
        """A gathered (all-gather-allocated) buffer left the live set: note when the compute stream is done with it."""
        if self.stage == 3 and self.is_cuda and self.groups[gi].P > 1 and not self.param_host \
                and self.cfg.gather_inflight_limit > 0 and not torch.cuda.is_current_stream_capturing():
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._free_events.append(ev)
            while len(self._free_events) > 4 * self.cfg.gather_inflight_limit:
                self._free_events.popleft()  # releases without new gathers (resident groups): keep the newest

    def _issue_gathers(self, gis) -> None:
        for gi in gis:
            self._issue_gather(gi)

    def fetch(self, gis) -> Dict[str, torch.Tensor]:
        out: Dict[str, torch.Tensor] = {}
        for gi in (gis if isinstance(gis, tuple) else (gis,)):
            self._issue_gather(gi)
            self._wait_update(gi)  # (P == 1: the views ARE the shard; wait where they are used, not at prefetch)
            flat, h = self._live[gi]
            h.wait()
            if self.param_host and self.is_cuda:
                flat.record_stream(torch.cuda.current_stream(self.device))  # allocated on the H2D stream
            views = self.groups[gi].views(flat)
            out.update(views)
            if gi in self._tnames:
                out.update(self._transposed(gi, views))
        return out

    def _transposed(self, gi: int, views: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """name + ".T" -> cached [in, out] copy of the stationary compute weight (rebuilt per step); expert-stacked
        [E, out, in] weights get [E, in, out] (one transpose per expert)."""
        ver, cache = self._tcache.get(gi, (-1, None))
        if cache is None:
            cache = {n: torch.empty(shp[:-2] + (shp[-1], shp[-2]), dtype=self.dtype, device=self.device)
                     for n, shp in self._tnames[gi]}
        if ver != self._pver:
            from ..ops.gemm import transpose
            from ..utils.streams import side_stream, test_delay
            # only the backward's input-gradient GEMMs read the copies: the rebuild (bandwidth-bound) runs on a side
            # stream beside the forward's compute and the group's next fetch (its backward visit) waits for it
            side = side_stream(self.device, "tcache") if self.is_cuda else None
            cur = torch.cuda.current_stream(self.device) if side is not None else None
            if side is not None:
                side.wait_stream(cur)
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                if side is not None:
                    test_delay()
                for n, shp in self._tnames[gi]:
                    if len(shp) == 3:
                        for e in range(shp[0]):
                            transpose(views[n][e], out=cache[n][e])
                    else:
                        transpose(views[n], out=cache[n])
            if side is not None:
                for n, _ in self._tnames[gi]:
                    views[n].record_stream(side)  # a gathered buffer may be released before the copies run
                ev = torch.cuda.Event()
                ev.record(side)
                self._tcache_ev[gi] = ev
            self._tcache[gi] = (self._pver, cache)
        else:
            ev = self._tcache_ev.pop(gi, None)
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
        return {n + ".T": t for n, t in cache.items()}

    def release(self, gis) -> None:
        if self.stage == 3:
            for gi in (gis if isinstance(gis, tuple) else (gis,)):
                if self._live.pop(gi, None) is not None:
                    self._released(gi)

    # ------------------------------------------------------------------ ZeRO-3 residency
    def _build_live_plan(self) -> None:
        """Visits of one micro-step (forward stages, then backward stages reversed) and the plan of
        which gathered groups stay resident between them (parallel/residency.py)."""
        n = len(self.stages)
        visits = [self.stages[si][1] for si in range(n)] + [self.stages[si][1] for si in range(n - 1, -1, -1)]
        gathered = [self.stage == 3 and g.P > 1 for g in self.groups]
        self._tcache_budget = lambda resident_bytes: math.inf  # noqa: E731
        hbm = lambda: math.inf  # noqa: E731
        if self.is_cuda:
            from .planner import zero3_budgets
            live, self._tcache_budget = zero3_budgets(
                torch.cuda.get_device_properties(self.device).total_memory, self._hbm_committed(gathered),
                self.cfg.live_hbm_fraction, self.cfg.tcache_hbm_fraction, self.cfg.hbm_headroom)
            hbm = lambda: live  # noqa: E731
        max_live = resolve_limit(self.cfg.max_live_parameters, hbm)
        max_reuse = resolve_limit(self.cfg.max_reuse_distance, hbm, unbounded_for_hbm=True)
        self.live_plan = ResidencyPlan(visits, [g.numel for g in self.groups], gathered, max_live, max_reuse)

    def _hbm_committed(self, gathered: List[bool]) -> float:
        """Bytes this rank will hold at its peak besides the optional ZeRO-3 residency / W^T caches: what is
        allocated now (shards, optimizer state, local gradients) + the planner's activation, scratch and
        in-flight-gather estimates (parallel/planner.py, the same rules it applies to a whole config)."""
        from .planner import _activation_bytes, runtime_reserve
        c = self.cfg
        now = float(torch.cuda.memory_allocated(self.device))
        extra = sum(_activation_bytes(self.mcfg, c.micro_batch_size * c.seq_len, c.seq_len,
                                      c.activation_checkpointing, self.ep_size).values())
        red = [g.numel for g in self.groups if g.P > 1]
        if self.stage in (2, 3) and red:
            extra += 4.0 * max(red) * (1 + 1.0 / self.W)
        sizes = sorted((sum(self.groups[gi].numel for gi in gis if gathered[gi]) for _, gis in self.stages),
                       reverse=True)
        if sizes:
            extra += 2.0 * (sizes[0] + (sizes[1] if len(sizes) > 1 else 0))
        return now + extra + runtime_reserve(now + extra)

    def _add_resident_tcache(self) -> None:
        """ZeRO-3, P > 1: a gathered group the residency plan holds through the whole step is as stationary
        between optimizer steps as a ZeRO-1/2 weight, so its dX GEMMs get the cached W^T as well (built on
        the first fetch after the step's all-gather, reused by every micro-batch). Without this a ZeRO-3
        run on N > 1 GPUs would lose the K-contiguous dX layout the single-GPU run has."""
        budget = self._tcache_budget(self.live_plan.resident_params * self.p16_shard.element_size())
        used = 0
        for g in self.groups:
            if g.P == 1 or g.idx in self._tnames or not self.live_plan.held_through_step(g.idx):
                continue
            names = [(sp.name, tuple(sp.shape)) for sp in g.specs if sp.tcache and len(sp.shape) == 2]
            nbytes = sum(shp[0] * shp[1] for _, shp in names) * self.p16_shard.element_size()
            if names and used + nbytes <= budget:
                self._tnames[g.idx] = names
                used += nbytes

    def _after_visit(self, v: int, gis, last_micro: bool) -> None:
        """Drop the gathered copies the residency plan does not keep past visit v (ZeRO-3)."""
        if self.stage == 3:
            for gi in gis:
                if not self.live_plan.keep(v, gi, last_micro):
                    if self._live.pop(gi, None) is not None:
                        self._released(gi)

    def _prefetch(self, si: int, step: int) -> None:
        """Issue the all-gathers of the stages after `si` (direction `step`): at least one stage, then
        more while the parameters in flight stay within prefetch_bucket_size (stage3_prefetch_bucket_size)."""
        if self.stage != 3 or not self.cfg.prefetch:
            return
        acc, j = 0, si + step
        while 0 <= j < len(self.stages):
            gis = self.stages[j][1]
            size = sum(self.groups[gi].numel for gi in gis if gi not in self._live and self.groups[gi].P > 1)
            if j != si + step and acc + size > self.cfg.prefetch_bucket_size:
                break
            self._issue_gathers(gis)
            acc += size
            j += step

    # ------------------------------------------------------------------ grads
    def _direct_target(self, g: FlatGroup) -> Optional[torch.Tensor]:
        """fp32 storage the unit backward writes / accumulates into directly, or None (bf16 scratch path).

        Direct whenever the group's gradient is not reduce-scattered per micro-batch: every group on
        a single rank (P == 1: the whole 1-GPU bench), ZeRO-0 (all-reduce at the boundary) and ZeRO-1
        (reduce-scatter of the local fp32 accumulator at the boundary). The weight-gradient GEMMs then
        run bf16 x bf16 -> fp32 with beta = 1 (ops.gemm.grad_mm): no bf16 rounding of per-micro-batch
        gradients, no scratch buffer and no separate accumulate pass.
        """
        if g.P == 1:
            # (raw partition, no join: a group is written only after its forward fetch waited for its update)
            return self._st_grad_shard.narrow(0, g.shard_off, g.shard_numel)
        if self.stage == 1 or self.local_grads:
            return self.grad_full.narrow(0, g.gfull_off, g.numel)
        return None

    def _post(self, g: FlatGroup) -> float:
        """Factor applied after group g's gradient reduction: 1 (AVG reductions) or, with
        prescale_gradients, predivide_factor / reduce world (SUM reductions of pre-divided gradients)."""
        if not self.cfg.prescale_gradients:
            return 1.0
        return self.cfg.gradient_predivide_factor / max(1, g.comm.world)

    def _finish_direct(self, g: FlatGroup, tgt: torch.Tensor, pending: List[Tuple[Handle, Any]]) -> None:
        """Boundary work for a direct group after its last backward visit of the last micro-batch."""
        if g.kind == "expert" and self.ep_size > 1:
            # an expert sees the tokens of every EP rank, each scaled by 1/(its own tokens): divide by the
            # EP size so expert grads are the global mean like the dense grads (which are AVG-reduced)
            tgt.mul_(1.0 / self.ep_size)
        avg, post = not self.cfg.prescale_gradients, self._post(g)
        step_dt = self.cfg.step_comm_dtype
        if (g.P > 1 and self.local_grads and step_dt in (torch.bfloat16, torch.float32) and tgt.dtype == torch.float32
                and self._mesh_ok(g, tgt)):
            # mesh: the fp32 accumulator is pushed as fp32 (or cast to bf16 on the fly); the reduce writes the shard
            shard_tgt = self._st_grad_shard.narrow(0, g.shard_off, g.shard_numel)
            scale = (1.0 / g.comm.world if avg else 1.0) * post
            m = self.mesh
            f32 = step_dt == torch.float32
            h = m.run_async(lambda: m.reduce_scatter(shard_tgt, tgt, scale, False, fp32=f32), [tgt, shard_tgt], "rs")
            pending.append((h, _Scaled(shard_tgt, 1.0, tgt)))
        elif g.P > 1 and self.local_grads and step_dt != tgt.dtype:
            # ZeRO-2/3 local accumulation, reduced in a 16-bit step_comm_dtype: half the bytes of fp32, then the
            # shard is written (beta = 0) from the reduced chunk
            src = tgt.to(step_dt)
            out = torch.empty(g.shard_numel, dtype=src.dtype, device=self.device)
            shard_tgt = self._st_grad_shard.narrow(0, g.shard_off, g.shard_numel)
            pending.append((g.comm.reduce_scatter(out, src, avg=avg, async_op=True),
                            (shard_tgt, out, 0.0, None, post, src)))
        elif g.P > 1:  # ZeRO-1, or fp32 step comm: reduce-scatter the local accumulator into this rank's shard
            out = self._st_grad_shard.narrow(0, g.shard_off, g.shard_numel)
            pending.append((g.comm.reduce_scatter(out, tgt, avg=avg, async_op=True), _Scaled(out, post, tgt)))
        elif g.comm.world > 1:  # ZeRO-0 / persistent (replicated) group: plain data parallel
            pending.append((g.comm.all_reduce(tgt, avg=avg, async_op=True), _Scaled(tgt, post)))
        elif post != 1.0:
            # no reduction for this group (W == 1, or an expert group at EP == W): the predivided gradient
            # still gets its post-scale (factor / 1), or it would stay 1/factor too small
            tgt.mul_(post)

    def _reduce_group_grad(self, gi: int, gbuf: torch.Tensor, first_micro: bool,
                           pending: List[Tuple[Handle, Any]]) -> None:
        """Scratch path (ZeRO-2/3, P > 1): reduce-scatter this micro-batch's bf16 gradient segment now."""
        g = self.groups[gi]
        beta = 0.0 if first_micro else 1.0
        alpha = (1.0 / self.ep_size if g.kind == "expert" else 1.0) * self._post(g)
        shard_tgt = self._st_grad_shard.narrow(0, g.shard_off, g.shard_numel)
        if gbuf.dtype == torch.bfloat16 and self.cfg.comm_dtype == torch.bfloat16 and self._mesh_ok(g, gbuf):
            scale = alpha * (1.0 / g.comm.world if not self.cfg.prescale_gradients else 1.0)
            m = self.mesh
            h = m.run_async(lambda: m.reduce_scatter(shard_tgt, gbuf, scale, beta == 1.0), [gbuf, shard_tgt], "rs")
            pending.append((h, _MeshRS(gbuf)))
            return
        src = gbuf
        if self.cfg.comm_dtype != gbuf.dtype:
            src = gbuf.to(self.cfg.comm_dtype)
            self._release_gbuf(gbuf)
        out = torch.empty(g.shard_numel, dtype=src.dtype, device=self.device)
        h = g.comm.reduce_scatter(out, src, avg=not self.cfg.prescale_gradients, async_op=True)
        pending.append((h, (shard_tgt, out, beta, src, alpha)))

    def _acquire_gbuf(self, numel: int) -> torch.Tensor:
        # flat bf16 gradient scratch, pooled per size and zeroed ONCE: units write only their
        # parameter ranges, so the ALIGN padding stays zero (garbage there would reach the
        # optimizer and trip the non-finite check)
        free = self._gbuf_pool.setdefault(numel, [])
        if free:
            return free.pop()
        return torch.zeros(numel, dtype=self.dtype, device=self.device)

    def _release_gbuf(self, buf: torch.Tensor) -> None:
        self._gbuf_pool.setdefault(buf.numel(), []).append(buf)

    def _drain(self, pending: List[Tuple[Handle, Any]], keep: int) -> None:
        while len(pending) > keep:
            h, payload = pending.pop(0)
            h.wait()
            if isinstance(payload, _Scaled):
                if payload.factor != 1.0:
                    payload.t.mul_(payload.factor)
            elif isinstance(payload, _MeshRS):
                self._release_gbuf(payload.src)  # the push has read it: back to the pool
            elif isinstance(payload, tuple):
                shard_tgt, out, beta, src, alpha = payload[:5]  # payload[5]: input kept alive until here
                ops.accumulate_(shard_tgt, out, alpha, beta)
                if src is not None and src.dtype == self.dtype:
                    self._release_gbuf(src)

    # ------------------------------------------------------------------ step
    def _context(self, ids: torch.Tensor, labels: torch.Tensor) -> StepContext:
        B, S = ids.shape
        gs = 1.0 / (B * S * self.cfg.grad_accum)
        if self.cfg.prescale_gradients:
            gs /= self.cfg.gradient_predivide_factor  # pre-divided before the SUM reductions
        return StepContext(batch=B, seq_len=S, input_ids=ids, labels=labels, grad_scale=gs, rope=self.rope,
                           ep_group=self.ep_comm, sp_group=self.sp_comm, ep_dispatcher=self.ep_mesh,
                           loss_scale=self.scaler.state[0:1] if self.scaler is not None else None)

    def micro_step(self, ids: torch.Tensor, labels: torch.Tensor, first: bool, last: bool) -> torch.Tensor:
        ctx = self._context(ids, labels)
        self._micro = 0 if first else getattr(self, "_micro", 0) + 1
        ctx.micro_index, ctx.last_micro = self._micro, last
        dw = self.cfg.defer_expert_wgrad
        ctx.defer_wgrad = bool((dw == "auto" and self.cfg.grad_accum > 1) or dw is True) and all(
            self._direct_target(g) is not None for g in self.groups if g.kind == "expert")
        ctx.defer_budget_bytes = int(self.cfg.defer_wgrad_budget_gb * (1 << 30))
        if last and self._xstats is not None:
            self._xstats.zero_()
            ctx.expert_stats = self._xstats  # units add each expert weight's final gradient statistics
        n = len(self.stages)
        saved: List[Any] = [None] * n
        x: Any = None
        ckpt = self.cfg.activation_checkpointing
        act = None
        if ckpt and self.cfg.cpu_checkpointing:
            if self._act_offload is None:
                from .offload import ActivationOffloader
                self._act_offload = ActivationOffloader(self.device)
            act = self._act_offload
        # ---- forward
        t_fwd = self.timers.mark()
        for si, (unit, gis) in enumerate(self.stages):
            p = self.fetch(gis)
            self._prefetch(si, +1)
            if ckpt and si < n - 1:
                y, _ = unit.forward(p, x, ctx)
                saved[si] = ("ckpt", act.push(x) if act is not None else x)
                if act is not None and si > 0:
                    saved[si - 1] = ("ckpt", act.release_device(saved[si - 1][1]))
            else:
                y, saved[si] = unit.forward(p, x, ctx)
            self._after_visit(si, gis, last)  # e.g. the head stays gathered for its backward right after
            x = y
        loss = x
        # ---- backward
        t_bwd = self.timers.mark()
        dy: Any = None
        pending: List[Tuple[Handle, Any]] = []
        gbufs: Dict[int, torch.Tensor] = {}
        visited: set = set()
        for si in range(n - 1, -1, -1):
            unit, gis = self.stages[si]
            p = self.fetch(gis)
            self._prefetch(si, -1)
            # per group: direct fp32 target or bf16 scratch, and whether this visit adds to what is there
            # (direct: any micro-batch after the first; both: the second visit of a tied group)
            gv: Dict[str, torch.Tensor] = {}
            want = {}
            for gi in gis:
                g = self.groups[gi]
                tgt = self._direct_target(g)
                if tgt is None:
                    if gi not in gbufs:
                        gbufs[gi] = self._acquire_gbuf(g.numel)
                    tgt = gbufs[gi]
                    want[gi] = gi in visited
                else:
                    want[gi] = gi in visited or not first
                gv.update(g.views(tgt))
            ctx.grad_acc = any(want.values())
            if ctx.grad_acc:
                for gi, w in want.items():  # mixed stage (e.g. direct experts + scratch dense): start from 0
                    if not w:
                        for v in self.groups[gi].views(gbufs[gi] if gi in gbufs else self._direct_target(
                                self.groups[gi])).values():
                            v.zero_()
            sv = saved[si]
            if isinstance(sv, tuple) and len(sv) == 2 and isinstance(sv[0], str) and sv[0] == "ckpt":
                xin = sv[1]
                if act is not None:
                    xin = act.get(xin)
                    if si > 0 and isinstance(saved[si - 1], tuple) and saved[si - 1][0] == "ckpt":
                        saved[si - 1] = ("ckpt", act.prefetch(saved[si - 1][1]))  # one unit ahead
                _, sv = unit.forward(p, xin, ctx)
            dy = unit.backward(p, gv, sv, dy, ctx)
            saved[si] = None
            visited.update(gis)
            if self.fault_inject_nan:
                next(iter(gv.values())).view(-1)[0] = float("nan")
                self.fault_inject_nan = False
            for gi in gis:
                if self._bwd_last_visit[gi] == si:
                    if gi in gbufs:
                        self._reduce_group_grad(gi, gbufs.pop(gi), first, pending)
                    elif last:
                        self._finish_direct(self.groups[gi], self._direct_target(self.groups[gi]), pending)
            self._after_visit(2 * n - 1 - si, gis, last)
            self._drain(pending, keep=1)
        self._drain(pending, keep=0)
        t_end = self.timers.mark()
        self.timers.span("forward", t_fwd, t_bwd)
        self.timers.span("backward+reduce", t_bwd, t_end)
        if self.stage == 3 and last:
            self._live.clear()  # nothing outlives the step: the optimizer changes the parameters
        self.last_aux = ctx.aux
        if last:  # every expert weight tallied by its final dW launch -> the optimizer skips their re-read
            self._xstats_ok = (self._xstats is not None
                               and ctx.aux.get("expert_stats_weights", 0) == self._xstats_weights)
        return loss

    def sync_params_from_master(self) -> None:
        """Recompute the bf16 compute copies from the fp32 master (after restore / external edits)."""
        self.join_optimizer()
        self._p16_from_master()
        if self.stage in (1, 2):
            hs = [self._all_gather(g, self.p16_full.narrow(0, g.full_off, g.numel), self._shard16(g))
                  for g in self.groups]
            for h in hs:
                h.wait()
        self._live.clear()

    def _global_grad_stats(self) -> None:
        """stats = [sum g^2, #non-finite, flags] over the whole model, each gradient element counted once;
        flags = sum over ranks of host_flag."""
        st = self.stats
        simple = not self.has_experts and (self.P == 1 or all(g.P > 1 for g in self.groups))
        if simple:
            ops.grad_stats([self.grad_shard], st)
            st[2].fill_(self.host_flag)
            if self.P > 1:
                self.comm.all_reduce(st, async_op=False).wait()
            elif self.sync_flags and self.W > 1:
                self.comm.all_reduce(st[2:3], async_op=False).wait()
        else:
            # partitioned dense groups: summed over ranks; replicated groups (ZeRO-0, persistent): counted
            # once; expert groups: summed over their expert-data-parallel and EP ranks
            sl = lambda g: self.grad_shard.narrow(0, g.shard_off, g.shard_numel)  # noqa: E731
            dense = torch.zeros(3, dtype=torch.float32, device=self.device)
            rep = torch.zeros(2, dtype=torch.float32, device=self.device)
            exp = torch.zeros(2, dtype=torch.float32, device=self.device)
            ops.grad_stats([sl(g) for g in self.groups if g.kind != "expert" and g.P > 1], dense)
            ops.grad_stats([sl(g) for g in self.groups if g.kind != "expert" and g.P == 1], rep)
            if self._xstats_ok:
                exp.copy_(self._xstats)
            else:
                ops.grad_stats([sl(g) for g in self.groups if g.kind == "expert"], exp)
            self._xstats_ok = False
            dense[2].fill_(self.host_flag)
            if any(g.P > 1 and g.kind != "expert" for g in self.groups):
                self.comm.all_reduce(dense, async_op=False).wait()
            elif self.sync_flags and self.W > 1:
                self.comm.all_reduce(dense[2:3], async_op=False).wait()
            if self.has_experts:
                if self.ep_comm is not None and self.ep_comm.world > 1:
                    self.ep_comm.all_reduce(exp, async_op=False).wait()
                eg = next(g for g in self.groups if g.kind == "expert")
                if eg.P > 1:
                    eg.comm.all_reduce(exp, async_op=False).wait()
            st.copy_(dense)
            st[:2] += rep + exp
        if self._nan_latch is not None:
            torch.maximum(self._nan_latch, st[1:2], out=self._nan_latch)
            st[1:2].copy_(self._nan_latch)

    def optimizer_step(self) -> Dict[str, Any]:
        t0 = self.timers.mark()
        out = self._optimizer_step()
        self.timers.span("optimizer_step", t0, self.timers.mark())
        return out

    def _optimizer_step(self) -> Dict[str, Any]:
        for hk in self.pre_step_hooks:
            hk(self)
        if self.param_nvme is not None:  # the partition file changes below: read-aheads in flight are stale
            self.param_nvme.drop_read_ahead()
        self.join_optimizer()
        self.step_count += 1
        cfg = self.cfg
        self._global_grad_stats()
        lr = lr_at(cfg, self.step_count)
        sst = self.scaler.state if self.scaler is not None else None
        # the step's gradient norm, unscaled on the device before the scaler moves on
        self.grad_norm = self.stats[0].sqrt() * sst[1] if sst is not None else self.stats[0].sqrt()
        if self.offload is not None:
            self._offload_step(lr, float(sst[1]) if sst is not None else 1.0)
        else:
            self._mesh_quiesce()
            if self._opt_overlap_ok():
                self._adamw_overlapped(lr, sst)
            else:
                ops.adamw_step_(self.master, self.exp_avg, self.exp_avg_sq, self.grad_shard,
                                None if self.param_host else self.p16_shard,
                                self.stats, lr=lr,
                                beta1=cfg.betas[0], beta2=cfg.betas[1], eps=cfg.eps, weight_decay=cfg.weight_decay,
                                step=self.step_count, grad_scale=1.0, max_norm=cfg.grad_clip, scale_state=sst)
            if self.param_host:
                self._p16_to_host()
            self._mesh_publish()
        self._pver += 1  # the compute copy changes below: transposed caches are stale
        if self.stage == 3:
            self._live.clear()  # (micro_step(last=True) already dropped them; direct callers may not have)
        if self.stage in (1, 2):
            hs = []
            for g in self.groups:
                hs.append(self._all_gather(g, self.p16_full.narrow(0, g.full_off, g.numel), self._shard16(g)))
            for h in hs:
                h.wait()
        if self.scaler is not None:
            self.scaler.update_(self.stats)
        return {"lr": lr, "stats": self.stats}

    def _opt_overlap_ok(self) -> bool:
        return (self.cfg.optimizer_overlap and self.is_cuda and self.stage == 3 and self.offload is None
                and not self.param_host and self.mesh is None)

    def _adamw_overlapped(self, lr: float, sst: Optional[torch.Tensor]) -> None:
        """cfg.optimizer_overlap: one AdamW launch per group on the optimizer stream, in forward order, each
        followed by an event that the group's next use waits on (_wait_update: at the gather of a partitioned group,
        at the fetch of an unpartitioned one). The statistics and the loss-scaler state are snapshotted first: the
        main stream moves on (scaler update, next step) at once. Measured +0.3 % on Mixtral 2-layer (the forward's
        GEMMs run at the board's power cap; profiles/optimizer_overlap_ab_r04.json)."""
        cfg = self.cfg
        if self._opt_stream is None:
            self._opt_stream = owned_stream(self.device, "optimizer", owner=self)
            self._opt_stats = torch.empty_like(self.stats)
            self._opt_sst = torch.empty_like(sst) if sst is not None else None
        self._opt_stats.copy_(self.stats)
        if sst is not None:
            self._opt_sst.copy_(sst)
        side = self._opt_stream
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            if self._opt_delay_cycles:
                torch.cuda._sleep(self._opt_delay_cycles)
            for gi in self._opt_order:
                g = self.groups[gi]
                if g.shard_numel > 0:
                    sl = lambda t: t.narrow(0, g.shard_off, g.shard_numel)  # noqa: E731
                    ops.adamw_step_(sl(self._st_master), sl(self._st_exp_avg), sl(self._st_exp_avg_sq),
                                    sl(self._st_grad_shard), sl(self._st_p16_shard), self._opt_stats, lr=lr, beta1=cfg.betas[0],
                                    beta2=cfg.betas[1], eps=cfg.eps, weight_decay=cfg.weight_decay,
                                    step=self.step_count, grad_scale=1.0, max_norm=cfg.grad_clip,
                                    scale_state=self._opt_sst)
                ev = torch.cuda.Event()
                ev.record(side)
                self._opt_pending[gi] = ev

    def _wait_update(self, gi: int) -> None:
        ev = self._opt_pending.pop(gi, None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)

    def join_optimizer(self) -> None:
        """The engine's compute stream AND the current stream wait for the overlapped optimizer updates still
        pending: anything that reads or writes master / moments / gradients / the compute copy outside the forward's
        fetches calls this (a state read under a side-stream context must not leave the compute stream unordered)."""
        if self._opt_pending:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(self._opt_stream)
            if self._compute_stream is not None and self._compute_stream != cur:
                self._compute_stream.wait_stream(self._opt_stream)
            self._opt_pending.clear()

    def _offload_step(self, lr: float, inv_scale: float) -> None:
        """Host AdamW over the offloaded partition; the clip / overflow decision needs the stats on the host
        (same formula as the device kernel, csrc/kernels/optim.hip clip_coef)."""
        cfg = self.cfg
        sumsq, nonfinite = (float(x) for x in self.stats[:2].tolist())
        if nonfinite > 0:
            return
        coef = inv_scale
        if cfg.grad_clip > 0:
            norm = math.sqrt(sumsq) * inv_scale
            coef *= min(1.0, cfg.grad_clip / (norm + 1e-6))
        self.offload.step(self.grad_shard, self.p16_shard, lr=lr, beta1=cfg.betas[0], beta2=cfg.betas[1],
                          eps=cfg.eps, weight_decay=cfg.weight_decay, step=self.step_count, gscale=coef)

    def train_step(self, micro_batches: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> Dict[str, Any]:
        """Run len(micro_batches) == grad_accum micro-batches and one optimizer step.

        Returns device tensors (``loss`` mean over the global batch of this rank,
        ``grad_norm``) -- nothing here synchronises with the host.
        """
        assert len(micro_batches) == self.cfg.grad_accum
        if self.graph_capturable() and not self.fault_inject_nan:
            self._graphed_micro_loop(micro_batches)
        else:
            self._micro_loop(micro_batches)
        out = self.optimizer_step()
        tokens = sum(int(ids.numel()) for ids, _ in micro_batches)
        metrics = {"loss": self.loss_acc / tokens, "grad_norm": self.grad_norm,
                   "nonfinite": self.stats[1], "lr": out["lr"], "step": self.step_count, "tokens": tokens}
        for hk in self.hooks:
            hk(self, metrics)
        return metrics

    def _micro_loop(self, micro_batches: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> None:
        self.loss_acc.zero_()
        for i, (ids, labels) in enumerate(micro_batches):
            loss = self.micro_step(ids, labels, first=(i == 0), last=(i == len(micro_batches) - 1))
            self.loss_acc += loss.float()

    # ------------------------------------------------------------------ HIP graphs
    def graph_capturable(self) -> bool:
        """Is the micro-batch loop free of collectives and host synchronisation (so it can be captured)?

        Single rank (every group P == 1: gradients land directly in the fp32 shard, no gather), a dense
        model or an MoE model on the grouped expert path at EP = 1 (the routing offsets stay on the device;
        the per-expert loop reads them on the host), no optimizer / activation offload (host copies), no
        per-phase timers (host-side event bookkeeping). The fp16 loss scale is a device word
        (LossScaler.state), so the fp16 path replays the same graph at every scale."""
        c = self.cfg
        moe_ok = not self.has_experts or self.ep_size == 1 or (self.ep_mesh is not None and not self.ep_mesh.sized)
        return (c.hip_graphs and self.is_cuda and (self.W == 1 or self._loop_on_mesh()) and moe_ok
                and self.offload is None
                and not self.param_host
                and not c.cpu_checkpointing and not self.timers.enabled
                and self.sp_size == 1 and self._graph_state != "failed")

    def _loop_on_mesh(self) -> bool:
        """W > 1: does every collective of the micro-batch loop ride the device-driven mesh (so the loop has
        no host-side collective and can be captured)? Dense groups partitioned over the world (gathers and
        bf16 reductions on the mesh), experts on their EP ranks only (EP == W: nothing to reduce), no
        replicated group (those all-reduce on RCCL), ZeRO-2/3."""
        if self.mesh is None or self.stage not in (2, 3) or self.cfg.comm_dtype != torch.bfloat16:
            return False
        if self.cfg.mesh_min_bytes > 0 or self.sp_size > 1:
            return False
        for g in self.groups:
            if g.kind == "expert":
                if g.P > 1 or g.comm.world > 1 or self.ep_mesh is None:
                    return False
            elif not self._mesh_group(g):
                return False
        return True

    def _graphed_micro_loop(self, micro_batches: Sequence[Tuple[torch.Tensor, torch.Tensor]]) -> None:
        """Capture the micro-batch loop once per batch shape (after one eager warm-up step that creates
        the library handles, hipBLASLt solutions and transposed-weight buffers), then replay it with the
        new token ids copied into the captured input buffers.

        The captured work writes only storage that outlives the graph (fp32 gradient shard, loss
        accumulator, the transposed-weight cache -- refreshed inside the graph at every replay, since
        its version is invalidated before the capture); activations live in the graph's private pool."""
        self.join_optimizer()  # (a captured wait on an event recorded outside the capture is not allowed)
        key = tuple((tuple(i.shape), tuple(l.shape)) for i, l in micro_batches)
        g = self._graph
        if g is None or g["key"] != key:
            if self._graph_state != "warm":  # first step of this shape: eager, creates lazy state
                self._graph_state = "warm"
                self._graph = None
                self._micro_loop(micro_batches)
                return
            static = [(i.clone(), l.clone()) for i, l in micro_batches]
            for gi in list(self._tcache):  # recompute the transposes inside the graph (stale each step)
                self._tcache[gi] = (-1, self._tcache[gi][1])
            self._graph = None
            torch.cuda.synchronize(self.device)
            self._tcache_ev.clear()  # (all side-stream rebuilds have run; a captured wait may not name them)
            torch.cuda.empty_cache()  # hand the eager step's cached activation blocks to the graph pool
            graph = torch.cuda.CUDAGraph()
            err = None
            try:
                with torch.cuda.graph(graph):
                    self._micro_loop(static)
            except Exception as e:  # an op that cannot be captured: stay eager for the rest of the run
                err = f"{type(e).__name__}: {e}"
            if self.W > 1:
                # every rank replays the same collective sequence: capture is all or nothing (host collective,
                # outside the captured region, once per batch shape)
                ok = torch.tensor([0.0 if err else 1.0], device=self.device)
                self.comm.all_reduce(ok, async_op=False).wait()
                if float(ok) < self.W and err is None:
                    err = "another rank could not capture its micro-batch loop"
            if err is not None:
                self._graph_state = "failed"
                self._tcache.clear()
                import warnings
                warnings.warn(f"HIP graph capture failed ({err}); running eagerly")
                torch.cuda.synchronize(self.device)
                self._micro_loop(micro_batches)
                return
            self._graph = {"key": key, "graph": graph, "static": static, "xstats_ok": self._xstats_ok}
            g = self._graph
        for (si, sl), (ids, labels) in zip(g["static"], micro_batches):
            if si.data_ptr() != ids.data_ptr():
                si.copy_(ids, non_blocking=True)
                sl.copy_(labels, non_blocking=True)
        g["graph"].replay()
        self._tcache = {gi: (self._pver, c) for gi, (_, c) in self._tcache.items()}
        # the captured loop's last micro-batch tallied the fused expert statistics iff it did at capture time
        self._xstats_ok = g["xstats_ok"]

    # ------------------------------------------------------------------ helpers
    def full_params(self) -> Dict[str, torch.Tensor]:
        """Gather all parameters (fp32 master) -- for tests / consolidated checkpoints.

        Expert tensors are concatenated over the expert-parallel ranks (global expert order).
        """
        return self._gather_flat(self.master)

    def full_grads(self) -> Dict[str, torch.Tensor]:
        """Gather the accumulated fp32 gradient partition (tests / debugging)."""
        return self._gather_flat(self.grad_shard)

    def _gather_flat(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {k: v for grp in self.iter_full(buf) for k, v in grp}

    def module_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """(name, full shape) of every parameter in iter_full order (experts: all EP ranks' experts)."""
        out = []
        epw = self.ep_comm.world if (self.ep_comm is not None and self.ep_comm.world > 1) else 1
        for g in self.groups:
            for s in g.specs:
                shp = tuple(s.shape)
                if g.kind == "expert" and epw > 1:
                    shp = (shp[0] * epw, *shp[1:])
                out.append((f"{g.prefix}.{s.name}", shp))
        return out

    def iter_full(self, buf: torch.Tensor, dtype: Optional[torch.dtype] = None):
        """Per group, the list of (name, full tensor) of flat state `buf` (master / grads): ZeRO shards
        all-gathered, expert tensors concatenated over the EP ranks (global expert order). Collective -- every
        rank runs the whole loop; one group is materialised at a time (checkpoint module capture streams it).
        `dtype`: cast the shard first (16-bit module state: half the gather bytes)."""
        self.join_optimizer()
        for g in self.groups:
            shard = buf.narrow(0, g.shard_off, g.shard_numel)
            if shard.device != self.device:  # offloaded optimizer state: collectives run on device tensors
                shard = shard.to(self.device)
            if dtype is not None and shard.dtype != dtype:
                shard = shard.to(dtype)
            if g.P > 1:
                full = torch.empty(g.numel, dtype=shard.dtype, device=self.device)
                g.comm.all_gather(full, shard, async_op=False).wait()
            else:
                full = shard
            items = []
            for k, v in g.views(full).items():
                v = v.clone()
                if g.kind == "expert" and self.ep_comm is not None and self.ep_comm.world > 1:
                    parts = torch.empty((self.ep_comm.world, *v.shape), dtype=v.dtype, device=v.device)
                    self.ep_comm.all_gather(parts.view(-1), v.reshape(-1), async_op=False).wait()
                    v = parts.reshape(-1, *v.shape[1:])
                items.append((f"{g.prefix}.{k}", v))
            yield items

    def memory_report(self) -> Dict[str, float]:
        gb = 1024 ** 3
        rep = {
            "optimizer_state_GiB": 0.0 if self.offload is not None else 3 * self.shard_total * 4 / gb,
            "optimizer_state_host_GiB": 3 * self.shard_total * 4 / gb if self.offload is not None else 0.0,
            "grad_shard_GiB": self.shard_total * 4 / gb,
            "param_shard_GiB": 0.0 if self.param_host else self.shard_total * 2 / gb,
            "param_shard_host_GiB": self.shard_total * 2 / gb if self.param_host else 0.0,
            "param_nvme_ring_GiB": (sum(t.numel() * t.element_size() for t in self.param_nvme.slots) / gb
                                    if self.param_nvme is not None else 0.0),
            "param_full_GiB": (self.full_total * 2 / gb) if self.p16_full is not None else 0.0,
            "grad_full_GiB": (self.gfull_total * 4 / gb) if self.grad_full is not None else 0.0,
            "weight_T_cache_GiB": sum(t.numel() * t.element_size() for _, c in self._tcache.values()
                                      for t in c.values()) / gb,
            "zero3_resident_gathered_GiB": self.live_plan.resident_params * self.p16_shard.element_size() / gb,
        }
        if self.is_cuda:
            rep["allocated_GiB"] = torch.cuda.memory_allocated(self.device) / gb
            rep["peak_GiB"] = torch.cuda.max_memory_allocated(self.device) / gb
        return rep

    def num_params(self) -> int:
        return sum(g.real_numel for g in self.groups)
