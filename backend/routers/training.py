"""Distributed-training endpoints (reference ``backend/routers/training.py``) + job supervision.

Same request models, defaults and responses for ``/launch``, ``/launch/preset``,
``/presets`` and ``/config/generate``. Fixes: an invalid offload device is a 422
(A16, enum-typed fields), ``/config/generate`` has no filesystem side effect
(A24). Additions: ``/jobs`` (registry of supervised launches), job cancel, and
``/jobs/{id}/preempt`` (spot-preemption drill: SIGUSR1 -> async emergency
checkpoint -> exit for restore).
"""
import signal
from typing import List, Optional

from fastapi import APIRouter, HTTPException
from pydantic import BaseModel, Field

from distributed_llm_training_gpu_manager_amd.launcher.config import (
    DeepSpeedConfig, LaunchResult, OffloadDevice, ZeROStage)
from distributed_llm_training_gpu_manager_amd.launcher.launcher import ZeroLauncher

router = APIRouter()
launcher = ZeroLauncher()


class TrainingLaunchRequest(BaseModel):
    training_script: str = Field(..., description="Path to training script")
    model_name: str = Field(default="custom_model")
    script_args: Optional[List[str]] = None
    zero_stage: int = Field(default=3, ge=0, le=3)
    offload_optimizer: OffloadDevice = Field(default=OffloadDevice.CPU)
    offload_param: OffloadDevice = Field(default=OffloadDevice.CPU)
    micro_batch_size: int = Field(default=4, ge=1)
    gradient_accumulation_steps: int = Field(default=8, ge=1)
    fp16: bool = True
    bf16: bool = False
    learning_rate: float = Field(default=3e-5, gt=0)
    warmup_steps: int = 100
    total_steps: int = 10000
    num_gpus: int = Field(default=1, ge=1)
    num_nodes: int = Field(default=1, ge=1)
    activation_checkpointing: bool = True
    dry_run: bool = Field(default=True, description="If true, only generates config without launching")


class PresetLaunchRequest(BaseModel):
    preset: str = Field(..., description="Preset name: 7b | 13b | 70b | gpt2-small | llama3-8b | llama3-70b | mixtral-8x7b")
    training_script: str = Field(...)
    script_args: Optional[List[str]] = None
    dry_run: bool = True


def _to_config(r: TrainingLaunchRequest) -> DeepSpeedConfig:
    return DeepSpeedConfig(
        model_name=r.model_name, zero_stage=ZeROStage(r.zero_stage), offload_optimizer=r.offload_optimizer,
        offload_param=r.offload_param, train_micro_batch_size_per_gpu=r.micro_batch_size,
        gradient_accumulation_steps=r.gradient_accumulation_steps, fp16_enabled=r.fp16, bf16_enabled=r.bf16,
        learning_rate=r.learning_rate, warmup_steps=r.warmup_steps, total_training_steps=r.total_steps,
        num_gpus=r.num_gpus, num_nodes=r.num_nodes, activation_checkpointing=r.activation_checkpointing)


@router.post("/launch", response_model=LaunchResult)
def launch_training(request: TrainingLaunchRequest):
    return launcher.launch(_to_config(request), request.training_script, request.script_args, request.dry_run)


@router.post("/launch/preset", response_model=LaunchResult)
def launch_from_preset(request: PresetLaunchRequest):
    presets = launcher.presets()
    if request.preset not in presets:
        raise HTTPException(status_code=400,
                            detail=f"Unknown preset '{request.preset}'. Available: {list(presets.keys())}")
    return launcher.launch(presets[request.preset], request.training_script, request.script_args, request.dry_run)


@router.get("/presets")
def list_presets():
    return {
        name: {
            "zero_stage": cfg.zero_stage.value,
            "offload_optimizer": cfg.offload_optimizer.value,
            "offload_param": cfg.offload_param.value,
            "micro_batch_size": cfg.train_micro_batch_size_per_gpu,
            "gradient_accumulation": cfg.gradient_accumulation_steps,
            "precision": "bf16" if cfg.bf16_enabled else "fp16",
            "num_gpus": cfg.num_gpus,
            "num_nodes": cfg.num_nodes,
            "activation_checkpointing": cfg.activation_checkpointing,
        }
        for name, cfg in presets_items()
    }


def presets_items():
    return launcher.presets().items()


@router.post("/config/generate")
def generate_config(request: TrainingLaunchRequest):
    config = _to_config(request)
    ds_config = launcher.generate_config(config)
    command = launcher.build_launch_command(config, request.training_script, request.script_args,
                                            config_path=launcher.default_config_path(config))
    return {"deepspeed_config": ds_config, "launch_command": command,
            "effective_batch_size": config.effective_batch_size}


@router.get("/jobs")
def list_jobs():
    jobs = launcher.registry.list()
    return {"total_jobs": len(jobs), "jobs": [j.to_dict() for j in jobs]}


@router.get("/jobs/{job_id}")
def get_job(job_id: str):
    job = launcher.registry.get(job_id)
    if job is None:
        raise HTTPException(status_code=404, detail=f"No job '{job_id}'")
    return job.to_dict()


@router.post("/jobs/{job_id}/cancel")
def cancel_job(job_id: str):
    if not launcher.registry.cancel(job_id):
        raise HTTPException(status_code=404, detail=f"No job '{job_id}'")
    return {"job_id": job_id, "status": "cancelling"}


@router.post("/jobs/{job_id}/preempt")
def preempt_job(job_id: str):
    """Spot-preemption drill: ranks receive SIGUSR1, write an async emergency checkpoint and exit."""
    if not launcher.registry.signal(job_id, signal.SIGUSR1):
        raise HTTPException(status_code=404, detail=f"No running job '{job_id}'")
    return {"job_id": job_id, "status": "preemption_signalled"}
