"""Model configurations (random-init architectures; no checkpoints are downloaded).

BASELINE.json names GPT-2-small, Llama-3 8B / 70B and Mixtral 8x7B; the
reference only names size presets (``ai_engine/deepspeed_launcher.py:369-407``)
without any architecture, so these are the public architectures of those
models.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace
from typing import Dict, Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str  # "llama" | "gpt2" | "mixtral"
    vocab_size: int
    d_model: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn_dim: int
    max_seq_len: int = 8192
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    n_experts: int = 0
    top_k: int = 2
    init_std: float = 0.02
    router_aux_coef: float = 0.02
    rope_scaling: Optional[dict] = field(default=None, compare=False)

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def qkv_dim(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    def num_params(self) -> int:
        D, F, V, L = self.d_model, self.ffn_dim, self.vocab_size, self.n_layers
        if self.arch == "gpt2":
            per = 4 * D * D + 4 * D + 2 * D * F + F + D + 4 * D
            return V * D + self.max_seq_len * D + L * per + 2 * D + (0 if self.tie_embeddings else V * D)
        attn = D * self.qkv_dim + self.n_heads * self.head_dim * D
        mlp = 3 * D * F * max(1, self.n_experts)
        router = D * self.n_experts if self.n_experts else 0
        per = attn + mlp + router + 2 * D
        return V * D + L * per + D + (0 if self.tie_embeddings else V * D)

    def active_params(self) -> int:
        """Parameters touched per token (MoE: top_k experts)."""
        if not self.n_experts:
            return self.num_params()
        D, F = self.d_model, self.ffn_dim
        return self.num_params() - self.n_layers * 3 * D * F * (self.n_experts - self.top_k)

    def flops_per_token(self, seq_len: int, recompute: bool = False) -> float:
        """Training FLOPs per token: 6*N_active (dense) + 6*L*S*D attention (causal: half of 12)."""
        dense = 6.0 * (self.active_params() - self.vocab_size * self.d_model)  # embedding lookup is free
        attn = 6.0 * self.n_layers * seq_len * self.n_heads * self.head_dim
        f = dense + attn
        if recompute:
            f += (dense + attn) / 3.0
        return f

    def to_dict(self) -> dict:
        return asdict(self)


PRESETS: Dict[str, ModelConfig] = {
    # GPT-2 small (124M); vocab padded 50257 -> 50304 for 128-byte aligned rows
    "gpt2-small": ModelConfig("gpt2-small", "gpt2", 50304, 768, 12, 12, 12, 3072, max_seq_len=1024,
                              norm_eps=1e-5, tie_embeddings=True),
    "llama3-8b": ModelConfig("llama3-8b", "llama", 128256, 4096, 32, 32, 8, 14336, max_seq_len=8192,
                             rope_theta=500000.0, norm_eps=1e-5),
    "llama3-70b": ModelConfig("llama3-70b", "llama", 128256, 8192, 80, 64, 8, 28672, max_seq_len=8192,
                              rope_theta=500000.0, norm_eps=1e-5),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", "mixtral", 32000, 4096, 32, 32, 8, 14336, max_seq_len=32768,
                                rope_theta=1e6, norm_eps=1e-5, n_experts=8, top_k=2),
    # Llama-3.2-1B shape (untied head): resilience drills that must fit a single box's scratch disk
    "llama3-1b": ModelConfig("llama3-1b", "llama", 128256, 2048, 16, 32, 8, 8192, max_seq_len=8192,
                             rope_theta=500000.0, norm_eps=1e-5),
    # small shapes for tests / smoke runs
    "llama-tiny": ModelConfig("llama-tiny", "llama", 512, 256, 2, 4, 2, 512, max_seq_len=256, rope_theta=10000.0),
    "llama-small": ModelConfig("llama-small", "llama", 32768, 1024, 4, 8, 8, 2816, max_seq_len=2048),
    "gpt2-tiny": ModelConfig("gpt2-tiny", "gpt2", 512, 128, 2, 2, 2, 512, max_seq_len=128, tie_embeddings=True),
    "mixtral-tiny": ModelConfig("mixtral-tiny", "mixtral", 512, 256, 2, 4, 2, 256, max_seq_len=256,
                                rope_theta=10000.0, n_experts=4, top_k=2),
}


def get_config(name: str, **overrides) -> ModelConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model '{name}'; available: {sorted(PRESETS)}")
    cfg = PRESETS[name]
    return replace(cfg, **overrides) if overrides else cfg
