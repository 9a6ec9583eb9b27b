"""Compat module: reference ``ai_engine/loss_monitor.py`` names."""
from distributed_llm_training_gpu_manager_amd.health.loss_monitor import (  # noqa: F401
    AlertSeverity, LossSpikeMonitor, MonitorConfig, MonitorState, SpikeAlert, TrainingMetrics)
