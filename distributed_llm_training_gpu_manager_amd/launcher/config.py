"""DeepSpeed-schema training configuration + generator (wire-compatible with the reference).

Mirrors ``ai_engine/deepspeed_launcher.py:22-100`` (enums, the 38-field
``DeepSpeedConfig``, ``LaunchResult``) and ``generate_config`` (``:114-240``) key
for key, so existing configs, presets and REST payloads keep working. The
generated JSON is *consumed by our own engine* (``train.py`` reads
``zero_optimization.*``, ``bf16``/``fp16``, ``optimizer``, ``scheduler``,
``gradient_clipping``, ``activation_checkpointing``) instead of DeepSpeed.

Documented deviations:
  * A20 -- ``communication_data_type`` follows the precision: a bf16 run with the
    default "fp16" comm type emits "bf16" (the reference sends fp16 grads in a bf16
    run);
  * A21 -- the elasticity block also carries ``micro_batch_sizes`` and ``version``;
  * A22 -- NVMe offload emits ``nvme_path``;
  * an extra ``"mi355x"`` block carries engine knobs DeepSpeed does not have
    (bucket policy, NaN trap, async checkpoint ring, attention kernel).
"""
from __future__ import annotations

from datetime import datetime, timezone
from enum import Enum
from typing import Any, Dict, Optional, Union

from pydantic import BaseModel, Field


class ZeROStage(int, Enum):
    DISABLED = 0
    OPTIMIZER_STATE = 1
    GRADIENT_PARTITIONING = 2
    FULL_PARTITIONING = 3


class OffloadDevice(str, Enum):
    NONE = "none"
    CPU = "cpu"
    NVME = "nvme"


def utcnow() -> datetime:
    return datetime.now(timezone.utc).replace(tzinfo=None)


class MI355XOptions(BaseModel):
    """Engine knobs with no DeepSpeed equivalent (emitted under the "mi355x" key)."""
    bucket_policy: str = Field(default="per_layer", description="per_layer | size")
    nan_trap: bool = True
    attention: str = Field(default="dlgm_flash", description="hand-written CDNA4 flash attention")
    checkpoint_interval: int = Field(default=0, ge=0, description="optimizer steps between async checkpoints")
    pinned_ring_gb: float = Field(default=0.0, ge=0, description="0 = size to one full shard snapshot")
    save_dir: Optional[str] = None
    shm_reserve: bool = Field(default=True, description="with save_dir: the supervisor reserves every rank's /dev/shm "
                              "snapshot file before the first launch (an early spot notice never waits for fresh "
                              "host pages) and keeps it across restarts")
    auto_resume: bool = True
    max_restarts: int = Field(default=3, ge=0)
    heartbeat_timeout_s: float = Field(
        default=-1.0, description="hung-rank detection: seconds without a rank heartbeat before the job is killed and "
        "resumed; -1 = auto (max(heartbeat_min_s, 10 x the steady step time)), 0 = off")
    heartbeat_min_s: float = Field(default=120.0, gt=0)
    startup_timeout_s: float = Field(default=900.0, gt=0,
                                     description="bound for a rank's first heartbeat (start-up, restore, first step)")
    comm_dtype: Optional[str] = None
    expert_parallel_size: int = Field(default=1, ge=1)
    sequence_parallel_size: int = Field(default=1, ge=1, description="Ulysses sequence parallelism (long context)")
    local_grad_accum: Union[bool, str] = Field(
        default="hbm", description="ZeRO-2/3: fp32 grads accumulate locally, one reduce-scatter per step ('hbm': if they fit)")
    hip_graphs: bool = Field(default=False, description="replay the micro-batch loop as one captured HIP graph "
                             "(single rank; or every collective on the xGMI mesh)")
    xgmi_mesh: str = Field(default="off", description="on: dense ZeRO gathers / reduce-scatters and the EP token "
                           "exchange over the device-driven xGMI mesh (HIP IPC symmetric heaps); off: RCCL rings")
    ep_capacity_factor: Optional[float] = Field(
        default=None, gt=0, description="mesh EP receive capacity, x the balanced share of rows; null = dropless "
        "(worst-case receive slot; a routing that overflows an explicit capacity stops the job)")
    auto_micro_batch: bool = Field(default=False, description="size the micro-batch (and GA, activation "
                                   "checkpointing) to the per-rank HBM plan, keeping the global batch")


class DeepSpeedConfig(BaseModel):
    """Configuration for ZeRO training (field names/defaults identical to the reference)."""
    # ZeRO configuration
    zero_stage: ZeROStage = ZeROStage.FULL_PARTITIONING
    offload_optimizer: OffloadDevice = OffloadDevice.CPU
    offload_param: OffloadDevice = OffloadDevice.CPU

    # Batch sizing
    train_micro_batch_size_per_gpu: int = Field(default=4, ge=1)
    gradient_accumulation_steps: int = Field(default=8, ge=1)
    gradient_clipping: float = Field(default=1.0, ge=0)

    # Precision
    fp16_enabled: bool = True
    bf16_enabled: bool = False
    fp16_loss_scale: float = 0
    fp16_loss_scale_window: int = 1000

    # Learning rate
    learning_rate: float = Field(default=3e-5, gt=0)
    lr_scheduler_type: str = "WarmupDecayLR"
    warmup_steps: int = 100
    total_training_steps: int = 10000

    # Communication
    communication_data_type: str = "fp16"
    prescale_gradients: bool = False
    gradient_predivide_factor: float = 1.0

    # Activation checkpointing
    activation_checkpointing: bool = True
    contiguous_memory_optimization: bool = True
    cpu_checkpointing: bool = False

    # ZeRO-3 specific
    stage3_max_live_parameters: int = 1_000_000_000
    stage3_max_reuse_distance: int = 1_000_000_000
    stage3_prefetch_bucket_size: int = 500_000_000
    stage3_param_persistence_threshold: int = 100_000
    stage3_gather_16bit_weights_on_model_save: bool = True
    reduce_bucket_size: int = 500_000_000

    # Advanced
    elastic_training: bool = False
    wall_clock_breakdown: bool = True
    dump_state: bool = False

    # Model info
    model_name: str = "custom_model"
    num_gpus: int = Field(default=1, ge=1)
    num_nodes: int = Field(default=1, ge=1)
    master_addr: str = "localhost"
    master_port: int = 29500

    # additions (not in the reference; defaults keep the reference JSON unchanged)
    nvme_path: Optional[str] = None
    mi355x: Optional[MI355XOptions] = None

    @property
    def precision(self) -> str:
        return "bf16" if self.bf16_enabled else "fp16" if self.fp16_enabled else "fp32"

    @property
    def effective_batch_size(self) -> int:
        return self.train_micro_batch_size_per_gpu * self.gradient_accumulation_steps * self.num_gpus * self.num_nodes


class LaunchResult(BaseModel):
    """Result of a launch (same fields as the reference ``LaunchResult``)."""
    job_id: str
    config_path: str
    command: str
    status: str = "launched"
    num_gpus: int
    num_nodes: int
    effective_batch_size: int
    timestamp: str = Field(default_factory=lambda: utcnow().isoformat())
    details: Dict[str, Any] = Field(default_factory=dict)


def generate_config(config: DeepSpeedConfig) -> Dict[str, Any]:
    """Emit the DeepSpeed JSON dict (same keys/values as the reference ``generate_config``)."""
    comm_dtype = config.communication_data_type
    if config.bf16_enabled and comm_dtype == "fp16":
        comm_dtype = "bf16"  # A20
    ds: Dict[str, Any] = {
        "train_micro_batch_size_per_gpu": config.train_micro_batch_size_per_gpu,
        "gradient_accumulation_steps": config.gradient_accumulation_steps,
        "gradient_clipping": config.gradient_clipping,
        "steps_per_print": 100,
        "wall_clock_breakdown": config.wall_clock_breakdown,
        "dump_state": config.dump_state,
        "zero_optimization": {
            "stage": config.zero_stage.value,
            "allgather_partitions": True,
            "allgather_bucket_size": config.reduce_bucket_size,
            "overlap_comm": True,
            "reduce_scatter": True,
            "reduce_bucket_size": config.reduce_bucket_size,
            "contiguous_gradients": True,
            "round_robin_gradients": True,
        },
        "scheduler": {
            "type": config.lr_scheduler_type,
            "params": {
                "warmup_min_lr": 0,
                "warmup_max_lr": config.learning_rate,
                "warmup_num_steps": config.warmup_steps,
                "total_num_steps": config.total_training_steps,
            },
        },
        "optimizer": {
            "type": "AdamW",
            "params": {"lr": config.learning_rate, "betas": [0.9, 0.999], "eps": 1e-8, "weight_decay": 0.01},
        },
        "communication_data_type": comm_dtype,
        "prescale_gradients": config.prescale_gradients,
        "gradient_predivide_factor": config.gradient_predivide_factor,
    }
    if config.bf16_enabled:
        ds["bf16"] = {"enabled": True}
    elif config.fp16_enabled:
        ds["fp16"] = {
            "enabled": True,
            "loss_scale": config.fp16_loss_scale,
            "loss_scale_window": config.fp16_loss_scale_window,
            "initial_scale_power": 16,
            "hysteresis": 2,
            "min_loss_scale": 1,
        }
    if config.zero_stage == ZeROStage.FULL_PARTITIONING:
        ds["zero_optimization"].update({
            "stage3_max_live_parameters": config.stage3_max_live_parameters,
            "stage3_max_reuse_distance": config.stage3_max_reuse_distance,
            "stage3_prefetch_bucket_size": config.stage3_prefetch_bucket_size,
            "stage3_param_persistence_threshold": config.stage3_param_persistence_threshold,
            "stage3_gather_16bit_weights_on_model_save": config.stage3_gather_16bit_weights_on_model_save,
            "sub_group_size": 1_000_000_000,
        })
    if config.offload_optimizer != OffloadDevice.NONE:
        off = {"device": config.offload_optimizer.value, "pin_memory": True, "buffer_count": 4, "fast_init": False}
        if config.offload_optimizer == OffloadDevice.NVME:
            off["nvme_path"] = config.nvme_path or "/local_nvme"  # A22
        ds["zero_optimization"]["offload_optimizer"] = off
    if config.offload_param != OffloadDevice.NONE:
        off = {"device": config.offload_param.value, "pin_memory": True, "buffer_count": 5,
               "buffer_size": 1_000_000_000, "max_in_cpu": 1_000_000_000}
        if config.offload_param == OffloadDevice.NVME:
            off["nvme_path"] = config.nvme_path or "/local_nvme"
        ds["zero_optimization"]["offload_param"] = off
    if config.activation_checkpointing:
        ds["activation_checkpointing"] = {
            "partition_activations": True,
            "cpu_checkpointing": config.cpu_checkpointing,
            "contiguous_memory_optimization": config.contiguous_memory_optimization,
            "number_checkpoints": None,
            "synchronize_checkpoint_boundary": False,
            "profile": False,
        }
    if config.elastic_training:
        mbs = config.train_micro_batch_size_per_gpu
        ds["elasticity"] = {
            "enabled": True,
            "max_train_batch_size": mbs * config.gradient_accumulation_steps * config.num_gpus * 2,
            "min_train_batch_size": mbs,
            "min_gpus": 1,
            "max_gpus": config.num_gpus * config.num_nodes,
            "prefer_larger_batch_size": True,
            "micro_batch_sizes": [mbs],  # A21
            "version": 0.2,
        }
    if config.mi355x is not None:
        ds["mi355x"] = config.mi355x.model_dump()
    return ds


def presets() -> Dict[str, DeepSpeedConfig]:
    """Reference presets (7b/13b/70b, ``deepspeed_launcher.py:369-407``) + MI355X presets.

    The MI355X presets drop CPU offload: with 288 GB of HBM per GPU the whole
    ZeRO-3 state of Llama-3-8B fits on ONE GPU and 70B fits on 8.
    """
    return {
        "7b": DeepSpeedConfig(model_name="7b_model", train_micro_batch_size_per_gpu=2, gradient_accumulation_steps=16,
                              zero_stage=ZeROStage.FULL_PARTITIONING, offload_optimizer=OffloadDevice.CPU,
                              offload_param=OffloadDevice.NONE, fp16_enabled=True, num_gpus=4),
        "13b": DeepSpeedConfig(model_name="13b_model", train_micro_batch_size_per_gpu=1, gradient_accumulation_steps=32,
                               zero_stage=ZeROStage.FULL_PARTITIONING, offload_optimizer=OffloadDevice.CPU,
                               offload_param=OffloadDevice.CPU, fp16_enabled=True, num_gpus=8),
        "70b": DeepSpeedConfig(model_name="70b_model", train_micro_batch_size_per_gpu=1, gradient_accumulation_steps=64,
                               zero_stage=ZeROStage.FULL_PARTITIONING, offload_optimizer=OffloadDevice.CPU,
                               offload_param=OffloadDevice.CPU, bf16_enabled=True, fp16_enabled=False,
                               activation_checkpointing=True, cpu_checkpointing=True, num_gpus=8, num_nodes=2),
        "gpt2-small": DeepSpeedConfig(model_name="gpt2-small", train_micro_batch_size_per_gpu=8,
                                      gradient_accumulation_steps=1, zero_stage=ZeROStage.OPTIMIZER_STATE,
                                      offload_optimizer=OffloadDevice.NONE, offload_param=OffloadDevice.NONE,
                                      bf16_enabled=True, fp16_enabled=False, activation_checkpointing=False,
                                      learning_rate=6e-4, warmup_steps=10, total_training_steps=1000, num_gpus=1),
        "llama3-8b": DeepSpeedConfig(model_name="llama3-8b", train_micro_batch_size_per_gpu=1,
                                     gradient_accumulation_steps=8, zero_stage=ZeROStage.FULL_PARTITIONING,
                                     offload_optimizer=OffloadDevice.NONE, offload_param=OffloadDevice.NONE,
                                     bf16_enabled=True, fp16_enabled=False, activation_checkpointing=False,
                                     num_gpus=8, mi355x=MI355XOptions()),
        "llama3-70b": DeepSpeedConfig(model_name="llama3-70b", train_micro_batch_size_per_gpu=1,
                                      gradient_accumulation_steps=16, zero_stage=ZeROStage.FULL_PARTITIONING,
                                      offload_optimizer=OffloadDevice.NONE, offload_param=OffloadDevice.NONE,
                                      bf16_enabled=True, fp16_enabled=False, activation_checkpointing=True,
                                      num_gpus=8, mi355x=MI355XOptions()),
        "mixtral-8x7b": DeepSpeedConfig(model_name="mixtral-8x7b", train_micro_batch_size_per_gpu=1,
                                        gradient_accumulation_steps=8, zero_stage=ZeROStage.FULL_PARTITIONING,
                                        offload_optimizer=OffloadDevice.NONE, offload_param=OffloadDevice.NONE,
                                        bf16_enabled=True, fp16_enabled=False, activation_checkpointing=True,
                                        num_gpus=8, mi355x=MI355XOptions(expert_parallel_size=8)),
    }
