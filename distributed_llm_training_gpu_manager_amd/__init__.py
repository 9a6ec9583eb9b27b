"""MI355X-native distributed LLM training orchestrator.

A from-scratch AMD Instinct MI355X (gfx950 / CDNA4) framework with the
capabilities of webspoilt/distributed-llm-training-gpu-manager: the FastAPI
control plane (``backend/``), DeepSpeed-schema ZeRO configs and presets
(:mod:`launcher`), an amdsmi GPU-health monitor (:mod:`health.gpu_manager`),
loss-spike / NaN detection (:mod:`health.loss_monitor`), spot resiliency and
auto-resume (:mod:`ckpt`) -- backed by our own engine: ZeRO-1/2/3 over RCCL
(:mod:`parallel`), hand-written HIP kernels (``csrc/kernels``, :mod:`ops`) and
explicit-backward model units (:mod:`models`).
"""
__version__ = "0.1.0"
