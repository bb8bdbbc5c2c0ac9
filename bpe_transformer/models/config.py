"""Model configuration and the named presets of the north-star configs.

Keys mirror the reference's LM config schema
(``tests/fixtures/ts_tests/model_config.json:1-12``): vocab_size,
context_length, d_model, num_layers, num_heads, d_ff, rope_theta and the
ablation flags remove_rmsnorm / use_post_norm / remove_rope / ffn_type.
``num_kv_heads`` (grouped-query attention) is an addition for the
Llama-style preset.
"""

from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from pathlib import Path


@dataclass
class ModelConfig:
    vocab_size: int = 10000
    context_length: int = 256
    d_model: int = 512
    num_layers: int = 4
    num_heads: int = 16
    d_ff: int = 1344
    rope_theta: float = 10000.0
    num_kv_heads: int | None = None
    remove_rmsnorm: bool = False
    use_post_norm: bool = False
    remove_rope: bool = False
    ffn_type: str | None = None
    eps: float = 1e-5
    extra: dict = field(default_factory=dict)

    @property
    def head_dim(self) -> int:
        return self.d_model // self.num_heads

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d.pop("extra")
        return d

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        known = {f.name for f in dataclasses.fields(cls)} - {"extra"}
        kw = {k: v for k, v in d.items() if k in known}
        extra = {k: v for k, v in d.items() if k not in known}
        return cls(**kw, extra=extra)

    @classmethod
    def from_json(cls, path: str | Path) -> "ModelConfig":
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def num_params(self, include_embedding: bool = True) -> int:
        d, f, L, V = self.d_model, self.d_ff, self.num_layers, self.vocab_size
        kv = (self.num_kv_heads or self.num_heads) * self.head_dim
        per_layer = d * d * 2 + 2 * d * kv + 2 * d
        per_layer += 3 * d * f if (self.ffn_type or "swiglu") == "swiglu" else 2 * d * f
        n = L * per_layer + d + V * d  # layers + ln_final + lm_head
        if include_embedding:
            n += V * d
        return n

    def train_flops_per_token(self, seq_len: int | None = None) -> float:
        """Model FLOPs per trained token: 6 * matmul params + causal attention (fwd+bwd)."""
        S = seq_len or self.context_length
        n = self.num_params(include_embedding=False) - self.d_model * (2 * self.num_layers + 1)
        attn = 6.0 * self.num_layers * S * self.d_model  # 12*L*S*d halved for causal
        return 6.0 * n + attn


# Named presets (BASELINE.json "configs").
PRESETS: dict[str, ModelConfig] = {
    # TinyStories ~17M plumbing config (4L/512d, RoPE+SwiGLU), seq 256, fp32 on CPU
    "tinystories-17m": ModelConfig(vocab_size=10000, context_length=256, d_model=512, num_layers=4, num_heads=16,
                                   d_ff=1344),
    # GPT-2-small shape with RoPE + SwiGLU + RMSNorm (the headline benchmark model)
    "gpt2-small": ModelConfig(vocab_size=50257, context_length=1024, d_model=768, num_layers=12, num_heads=12,
                              d_ff=2048),
    # Llama-style 1.1B (TinyLlama shape: 22L/2048d, 32 q heads / 4 kv heads, SwiGLU 5632)
    "llama-1.1b": ModelConfig(vocab_size=32000, context_length=2048, d_model=2048, num_layers=22, num_heads=32,
                              num_kv_heads=4, d_ff=5632),
    # the reference test-suite model (tests/fixtures/ts_tests/model_config.json)
    "ts-tests": ModelConfig(vocab_size=10000, context_length=16, d_model=64, num_layers=3, num_heads=4, d_ff=128),
}


def get_preset(name: str, **overrides) -> ModelConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; have {sorted(PRESETS)}")
    cfg = dataclasses.replace(PRESETS[name])
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg
