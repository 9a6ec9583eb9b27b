"""Model zoo: GPT-2, Llama-3 (8B/70B), Mixtral 8x7B -- random init, explicit-backward units."""
from .config import ModelConfig, PRESETS, get_config
from .common import ParamSpec, StepContext, Unit, AutogradUnit


def build_model(cfg: ModelConfig, ep_rank: int = 0, ep_size: int = 1):
    """Return ``(param_groups, stages)`` for the engine.

    param_groups: list of (name, [ParamSpec]) -- one flat ZeRO segment each.
    stages: list of (unit, group_index) in forward order (a group may appear twice: tied weights).
    """
    if cfg.arch == "llama":
        from .llama import build
    elif cfg.arch == "gpt2":
        from .gpt2 import build
    elif cfg.arch == "mixtral":
        from .mixtral import build
        return build(cfg, ep_rank, ep_size)
    else:
        raise ValueError(f"unknown arch {cfg.arch}")
    return build(cfg)


__all__ = ["ModelConfig", "PRESETS", "get_config", "ParamSpec", "StepContext", "Unit", "AutogradUnit", "build_model"]
