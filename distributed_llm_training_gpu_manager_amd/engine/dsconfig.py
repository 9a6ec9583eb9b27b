"""Consume a DeepSpeed-schema JSON (as emitted by :func:`launcher.config.generate_config`) into EngineConfig.

Every key the reference's generator writes (``ai_engine/deepspeed_launcher.py:124-238``)
is either honoured or explicitly reported as not applicable on MI355X.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Tuple, Union

import torch

from ..parallel.zero import EngineConfig


def engine_config_from_ds(ds: Union[str, Dict[str, Any]], seq_len: int, model_cfg=None, world: int = 1,
                          **overrides) -> Tuple[EngineConfig, List[str]]:
    """``model_cfg`` / ``world``: needed only to resolve ``"train_micro_batch_size_per_gpu": "auto"`` (or
    the ``mi355x.auto_micro_batch`` switch) through the per-rank HBM planner."""
    if isinstance(ds, str):
        with open(ds) as f:
            ds = json.load(f)
    notes: List[str] = []
    mi = ds.get("mi355x") or {}
    auto_mbs = ds.get("train_micro_batch_size_per_gpu") == "auto" or bool(mi.get("auto_micro_batch", False))
    zo = ds.get("zero_optimization", {})
    opt = ds.get("optimizer", {}).get("params", {})
    sch = ds.get("scheduler", {})
    sp = sch.get("params", {})
    fp16 = ds.get("fp16", {}).get("enabled", False)
    bf16 = ds.get("bf16", {}).get("enabled", False)
    comm = ds.get("communication_data_type", "bf16")
    comm_dtype = {"fp32": torch.float32, "float32": torch.float32}.get(comm, torch.bfloat16)
    if comm in ("fp16", "float16"):
        notes.append("communication_data_type fp16 mapped to bf16 (A20)")
    off_o = zo.get("offload_optimizer", {}).get("device", "none")
    off_p = zo.get("offload_param", {}).get("device", "none")
    if off_p != "none" and int(zo.get("stage", 0)) != 3:
        notes.append(f"offload_param={off_p} needs ZeRO-3 (as in DeepSpeed): parameters stay in HBM")
    act = ds.get("activation_checkpointing")
    cfg = EngineConfig(
        zero_stage=int(zo.get("stage", 0)),
        micro_batch_size=1 if auto_mbs else int(ds.get("train_micro_batch_size_per_gpu", 1)),
        seq_len=seq_len,
        grad_accum=int(ds.get("gradient_accumulation_steps", 1)),
        lr=float(opt.get("lr", sp.get("warmup_max_lr", 3e-5))),
        betas=tuple(opt.get("betas", (0.9, 0.999))),
        eps=float(opt.get("eps", 1e-8)),
        weight_decay=float(opt.get("weight_decay", 0.01)),
        grad_clip=float(ds.get("gradient_clipping", 0.0)),
        scheduler=sch.get("type", "constant"),
        warmup_steps=int(sp.get("warmup_num_steps", 0)),
        total_steps=int(sp.get("total_num_steps", 10 ** 9)),
        warmup_min_lr=float(sp.get("warmup_min_lr", 0.0)),
        warmup_type=sp.get("warmup_type", "log"),
        comm_dtype=comm_dtype,
        activation_checkpointing=bool(act),
        cpu_checkpointing=bool(act and act.get("cpu_checkpointing", False)),
        fp16=bool(fp16 and not bf16),
        loss_scale=float(ds.get("fp16", {}).get("loss_scale", 0.0)),
        initial_scale_power=int(ds.get("fp16", {}).get("initial_scale_power", 16)),
        loss_scale_window=int(ds.get("fp16", {}).get("loss_scale_window", 1000)),
        hysteresis=int(ds.get("fp16", {}).get("hysteresis", 2)),
        min_loss_scale=float(ds.get("fp16", {}).get("min_loss_scale", 1.0)),
        offload_optimizer=off_o,
        nvme_path=zo.get("offload_optimizer", {}).get("nvme_path") or zo.get("offload_param", {}).get("nvme_path"),
        param_nvme_path=zo.get("offload_param", {}).get("nvme_path"),
        offload_buffer_count=int(zo.get("offload_optimizer", {}).get("buffer_count", 4)),
        aio_threads=max(1, int(ds.get("aio", {}).get("thread_count", 1)) * int(ds.get("aio", {}).get("queue_depth", 8))),
        aio_block_size=int(ds.get("aio", {}).get("block_size", 8 << 20)),
        wall_clock_breakdown=bool(ds.get("wall_clock_breakdown", False)),
        # ZeRO-3 residency (parallel/residency.py); a number, or "hbm" to size the budget to the GPU
        max_live_parameters=zo.get("stage3_max_live_parameters", 1e9),
        max_reuse_distance=zo.get("stage3_max_reuse_distance", 1e9),
        prefetch_bucket_size=float(zo.get("stage3_prefetch_bucket_size", 5e8)),
        param_persistence_threshold=float(zo.get("stage3_param_persistence_threshold", 0.0)),
        prescale_gradients=bool(ds.get("prescale_gradients", False)),
        gradient_predivide_factor=float(ds.get("gradient_predivide_factor", 1.0)),
        offload_param=off_p,
        param_buffer_count=int(zo.get("offload_param", {}).get("buffer_count", 5)),
        # DeepSpeed's default is False: without the key a stage-3 save carries no gathered 16-bit module
        gather_16bit_weights_on_model_save=bool(zo.get("stage3_gather_16bit_weights_on_model_save", False)),
    )
    # engine knobs without a DeepSpeed key travel in the "mi355x" block (launcher.config.MI355XOptions)
    cfg.expert_parallel_size = int(mi.get("expert_parallel_size", cfg.expert_parallel_size))
    cfg.sequence_parallel_size = int(mi.get("sequence_parallel_size", cfg.sequence_parallel_size))
    if "local_grad_accum" in mi:
        cfg.local_grad_accum = mi["local_grad_accum"]
    if "hip_graphs" in mi:
        cfg.hip_graphs = bool(mi["hip_graphs"])
    if "xgmi_mesh" in mi:
        v = mi["xgmi_mesh"]
        cfg.xgmi_mesh = ("on" if v else "off") if isinstance(v, bool) else str(v)
    if "ep_capacity_factor" in mi:
        v = mi["ep_capacity_factor"]
        cfg.ep_capacity_factor = None if v in (None, "dropless", "auto") else float(v)
    if mi.get("comm_dtype"):
        cfg.comm_dtype = {"fp32": torch.float32, "float32": torch.float32}.get(mi["comm_dtype"], torch.bfloat16)
    if mi.get("step_comm_dtype"):  # the once-per-step reduce of the local fp32 accumulator (default fp32)
        cfg.step_comm_dtype = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16}.get(mi["step_comm_dtype"],
                                                                                      torch.float32)
    if auto_mbs:
        _auto_micro_batch(cfg, ds, model_cfg, world, notes)
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg, notes


def _auto_micro_batch(cfg: EngineConfig, ds: Dict[str, Any], model_cfg, world: int, notes: List[str]) -> None:
    """Resolve the micro-batch (and gradient accumulation, activation checkpointing) from the planner,
    keeping the global batch: ``train_batch_size`` if given, else the configured mbs x GA x world."""
    if model_cfg is None:
        notes.append("train_micro_batch_size_per_gpu=auto needs the model: micro-batch 1")
        return
    from ..parallel.planner import auto_micro_batch

    mbs = ds.get("train_micro_batch_size_per_gpu")
    mbs = int(mbs) if isinstance(mbs, (int, float)) else 1
    sp = max(1, cfg.sequence_parallel_size)
    dp = max(1, world // sp)
    gb = ds.get("train_batch_size")
    gb = int(gb) if isinstance(gb, (int, float)) else mbs * cfg.grad_accum * dp
    ch = auto_micro_batch(model_cfg, world=world, data_parallel=dp, seq_len=cfg.seq_len // sp, global_batch=gb,
                          zero_stage=cfg.zero_stage,
                          ep_size=cfg.expert_parallel_size, offload_optimizer=cfg.offload_optimizer,
                          offload_param=cfg.offload_param, force_checkpointing=cfg.activation_checkpointing,
                          allow_checkpointing=True)
    cfg.micro_batch_size, cfg.grad_accum = ch.micro_batch, ch.grad_accum
    cfg.activation_checkpointing = ch.activation_checkpointing
    notes.append(f"auto micro-batch: {ch.micro_batch} x GA {ch.grad_accum} x {dp} ranks = {gb} sequences/step, "
                 f"checkpointing {'on' if ch.activation_checkpointing else 'off'}, planned "
                 f"{ch.plan.total / 2**30:.1f} GiB/rank (headroom {ch.plan.headroom:.0%})")
