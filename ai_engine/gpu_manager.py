"""Compat module: reference ``ai_engine/gpu_manager.py`` names -> amdsmi-backed MI355X implementation."""
from distributed_llm_training_gpu_manager_amd.health.gpu_manager import (  # noqa: F401
    GPUDevice, GPUFleetStatus, GPUHealthStatus, GPUManager, GPUProcess, XGMILink)
