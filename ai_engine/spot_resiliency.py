"""Compat module: reference ``ai_engine/spot_resiliency.py`` name -> working preemption manager."""
from distributed_llm_training_gpu_manager_amd.ckpt.spot import SpotInstanceResiliencyManager  # noqa: F401
