"""Fused MI355X ops. GPU tensors -> hand-written HIP kernels (csrc/kernels); CPU -> fp32 reference."""
from .norm import rmsnorm, rmsnorm_fwd, rmsnorm_bwd, RMSNormFunction
from .rope import rope_, rope_tables
from .activation import swiglu_fwd, swiglu_bwd
from .attention import flash_attn_fwd, flash_attn_bwd, flash_attention, flash_attention_qkv
from .loss import cross_entropy_fwd_bwd_
from .optim import grad_stats, adamw_step_, accumulate_, cast_f32_bf16_, loss_scale_update_
from .embedding import embedding_fwd, embedding_bwd_
from .moe import router_topk, moe_permute, moe_combine, moe_combine_bwd

__all__ = [
    "rmsnorm", "rmsnorm_fwd", "rmsnorm_bwd", "RMSNormFunction", "rope_", "rope_tables", "swiglu_fwd",
    "swiglu_bwd", "flash_attn_fwd", "flash_attn_bwd", "flash_attention", "flash_attention_qkv", "cross_entropy_fwd_bwd_",
    "grad_stats", "adamw_step_", "loss_scale_update_", "accumulate_", "cast_f32_bf16_", "embedding_fwd", "embedding_bwd_",
    "router_topk", "moe_permute", "moe_combine", "moe_combine_bwd",
]
