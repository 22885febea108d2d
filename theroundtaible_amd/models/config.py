"""Model architecture presets (SURVEY §2.4.1 shape table)."""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Dict, Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str                 # "llama" (Llama-3 / Mistral / Qwen2) | "gpt2"
    n_layers: int
    hidden: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn: int
    vocab: int
    max_pos: int
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    qkv_bias: bool = False    # Qwen2 / Qwen2.5: biased q/k/v projections (added before RoPE)
    # checkpoint RoPE scaling (ops/reference.py rope_inv_freq): ("linear", f) | ("llama3", f, low,
    # high, original_max_pos) | ("yarn", f, original_max_pos, beta_fast, beta_slow, attention_factor)
    rope_scaling: Optional[tuple] = None

    @property
    def q_size(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.n_kv_heads * self.head_dim

    @property
    def group(self) -> int:
        return self.n_heads // self.n_kv_heads

    def n_params(self) -> int:
        h, f, v, L = self.hidden, self.ffn, self.vocab, self.n_layers
        if self.arch == "gpt2":
            per = 4 * h * h + 2 * h * f + 9 * h + f
            return L * per + v * h + self.max_pos * h + 2 * h
        per = h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * f + 2 * h
        if self.qkv_bias:
            per += self.q_size + 2 * self.kv_size
        emb = v * h * (1 if self.tie_embeddings else 2)
        return L * per + emb + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * self.n_kv_heads * self.head_dim * dtype_bytes


PRESETS: Dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig("llama3-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256, 131072, 500000.0, 1e-5),
    # Llama 3.1 / 3.2: the same blocks with rope_type "llama3" scaling (3.2: tied embeddings;
    # 3.2-3B has GQA group 3)
    "llama3.1-8b": ModelConfig("llama3.1-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256, 131072, 500000.0, 1e-5,
                               False, False, ("llama3", 8.0, 1.0, 4.0, 8192)),
    "llama3.2-1b": ModelConfig("llama3.2-1b", "llama", 16, 2048, 32, 8, 64, 8192, 128256, 131072, 500000.0, 1e-5,
                               True, False, ("llama3", 32.0, 1.0, 4.0, 8192)),
    "llama3.2-3b": ModelConfig("llama3.2-3b", "llama", 28, 3072, 24, 8, 128, 8192, 128256, 131072, 500000.0, 1e-5,
                               True, False, ("llama3", 32.0, 1.0, 4.0, 8192)),
    "llama3-70b": ModelConfig("llama3-70b", "llama", 80, 8192, 64, 8, 128, 28672, 128256, 131072, 500000.0, 1e-5),
    "mistral-7b": ModelConfig("mistral-7b", "llama", 32, 4096, 32, 8, 128, 14336, 32000, 32768, 1000000.0, 1e-5),
    # Qwen2.5 (HF model_type "qwen2"): the Llama block with q/k/v biases; 7B: GQA 28 / 4 heads,
    # 0.5B: head_dim 64, tied embeddings (the family most local coding setups run)
    "qwen2.5-7b": ModelConfig("qwen2.5-7b", "llama", 28, 3584, 28, 4, 128, 18944, 152064, 32768, 1000000.0, 1e-6,
                              False, True),
    "qwen2.5-14b": ModelConfig("qwen2.5-14b", "llama", 48, 5120, 40, 8, 128, 13824, 152064, 32768, 1000000.0, 1e-6,
                               False, True),
    "qwen2.5-32b": ModelConfig("qwen2.5-32b", "llama", 64, 5120, 40, 8, 128, 27648, 152064, 32768, 1000000.0, 1e-6,
                               False, True),
    "qwen2.5-72b": ModelConfig("qwen2.5-72b", "llama", 80, 8192, 64, 8, 128, 29568, 152064, 32768, 1000000.0, 1e-6,
                               False, True),
    "qwen2.5-0.5b": ModelConfig("qwen2.5-0.5b", "llama", 24, 896, 14, 2, 64, 4864, 151936, 32768, 1000000.0, 1e-6,
                                True, True),
    # GPT-2-small: random init allows n_positions beyond 1024 (SURVEY §7.3 hard part 3).
    "gpt2-small": ModelConfig("gpt2-small", "gpt2", 12, 768, 12, 12, 64, 3072, 50257, 8192, 0.0, 1e-5, True),
    # test-sized models (CPU unit tests, GPU smoke)
    "tiny-llama": ModelConfig("tiny-llama", "llama", 2, 256, 4, 2, 64, 512, 32000, 4096, 10000.0, 1e-5),
    "tiny-llama-128": ModelConfig("tiny-llama-128", "llama", 2, 512, 4, 1, 128, 1024, 32000, 8192, 500000.0, 1e-5),
    "tiny-qwen": ModelConfig("tiny-qwen", "llama", 2, 256, 4, 2, 64, 512, 32000, 4096, 1000000.0, 1e-6, True, True),
    "tiny-qwen-128": ModelConfig("tiny-qwen-128", "llama", 2, 512, 4, 1, 128, 1024, 32000, 8192, 1000000.0, 1e-6,
                                 False, True),
    "tiny-gpt2": ModelConfig("tiny-gpt2", "gpt2", 2, 128, 2, 2, 64, 512, 32000, 2048, 0.0, 1e-5, True),
}


def get_config(name: str, **overrides) -> ModelConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset '{name}' (known: {', '.join(PRESETS)})")
    cfg = PRESETS[name]
    if isinstance(overrides.get("rope_scaling"), list):   # from a JSON config
        overrides = dict(overrides, rope_scaling=tuple(overrides["rope_scaling"]))
    return replace(cfg, **overrides) if overrides else cfg
