"""Compat module: reference ``ai_engine/deepspeed_launcher.py`` names -> the in-house ZeRO launcher."""
from distributed_llm_training_gpu_manager_amd.launcher.config import (  # noqa: F401
    DeepSpeedConfig, LaunchResult, MI355XOptions, OffloadDevice, ZeROStage, generate_config, presets)
from distributed_llm_training_gpu_manager_amd.launcher.launcher import DeepSpeedLauncher, ZeroLauncher  # noqa: F401
