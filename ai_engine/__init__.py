"""Drop-in import compatibility with the reference's ``ai_engine`` package.

The reference exposes ``GPUManager, GPUDevice, GPUFleetStatus, DeepSpeedLauncher,
DeepSpeedConfig, LossSpikeMonitor, TrainingMetrics, SpikeAlert`` (``ai_engine/__init__.py:9-17``).
Code written against it keeps working: every name resolves to the MI355X-native
implementation in :mod:`distributed_llm_training_gpu_manager_amd`.
"""
from distributed_llm_training_gpu_manager_amd.health.gpu_manager import GPUDevice, GPUFleetStatus, GPUManager
from distributed_llm_training_gpu_manager_amd.health.loss_monitor import LossSpikeMonitor, SpikeAlert, TrainingMetrics
from distributed_llm_training_gpu_manager_amd.launcher.config import DeepSpeedConfig
from distributed_llm_training_gpu_manager_amd.launcher.launcher import DeepSpeedLauncher

__all__ = [
    "GPUManager", "GPUDevice", "GPUFleetStatus",
    "DeepSpeedLauncher", "DeepSpeedConfig",
    "LossSpikeMonitor", "TrainingMetrics", "SpikeAlert",
]
