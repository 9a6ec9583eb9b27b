"""Training-loop plumbing around the ZeRO engine: DeepSpeed-JSON bridge, data, trainer."""
