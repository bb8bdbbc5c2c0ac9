"""Training configuration (dataclasses, JSON-loadable, CLI-overridable).

The reference has no training loop ("absent layers"); the
schema here covers what its utilities imply (``tests/adapters.py:401-542``):
batch sampling, AdamW, cosine LR with warmup, gradient clipping and
checkpointing -- plus data parallelism and mixed precision for MI355X.
"""

from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from pathlib import Path

from ..models.config import ModelConfig, get_preset


@dataclass
class OptimConfig:
    lr: float = 3e-4
    min_lr: float = 3e-5
    warmup_iters: int = 100
    cosine_cycle_iters: int | None = None  # default: max_iters
    betas: tuple[float, float] = (0.9, 0.95)
    eps: float = 1e-8
    weight_decay: float = 0.1
    max_grad_norm: float | None = 1.0


@dataclass
class DataConfig:
    train_path: str | None = None  # flat uint16/uint32 token file (np.memmap); None = synthetic
    val_path: str | None = None
    vocab_size_for_dtype: int = 65536
    synthetic_tokens: int = 1 << 22


@dataclass
class TrainConfig:
    model: ModelConfig = field(default_factory=lambda: get_preset("tinystories-17m"))
    optim: OptimConfig = field(default_factory=OptimConfig)
    data: DataConfig = field(default_factory=DataConfig)
    batch_size: int = 32  # per-device micro-batch (sequences)
    grad_accum: int = 1
    max_iters: int = 1000
    seed: int = 1234
    device: str = "auto"  # auto | cuda | cpu
    dtype: str = "auto"  # auto (bf16 on GPU, fp32 on CPU) | bf16 | fp32
    precision: str = "default"  # default | fp8 (block projections' forward GEMMs in e4m3, delayed scaling; GPU)
    bucket_mb: float = 64.0
    log_every: int = 10
    eval_every: int = 0
    eval_iters: int = 20
    ckpt_every: int = 0
    ckpt_dir: str = "output/checkpoints"
    resume: str | None = None  # path or "latest"
    metrics_path: str | None = None  # JSONL
    profile: bool = False
    phase_timing: bool = False  # log fwd / bwd / exposed-comm / optimizer ms (device events) at each log step
    nan_guard: bool = True
    ddp_check_every: int = 0  # >0: every N steps assert bit-identical grads / weights across DP ranks
    zero: int = 0  # 1: sharded data parallelism (reduce-scatter + 1/N AdamW + all-gather, parallel/zero.py)
    # flat gradient buffer dtype: auto (fp32 when grad_accum > 1, so the micro-batch sum is not rounded to bf16
    # every add; else the parameter dtype) | bf16 | fp32
    grad_dtype: str = "auto"
    comm_dtype: str = "auto"  # data-parallel all-reduce dtype: auto (= grad dtype) | bf16 | fp32
    # LM head + CE (ops/loss.py): logits (one [tokens, vocab] buffer, fastest) | streamed (token chunks of
    # lm_head_chunk rows, dh / dW formed in the forward: memory O(chunk * vocab)); lm_head_chunk 0 = default
    lm_head_mode: str = "logits"
    lm_head_chunk: int = 0

    def resolved_grad_dtype(self, param_dtype):
        import torch

        if self.grad_dtype == "auto":
            return torch.float32 if (self.grad_accum > 1 and param_dtype == torch.bfloat16) else None
        return {"bf16": torch.bfloat16, "fp32": torch.float32}[self.grad_dtype]

    def resolved_comm_dtype(self):
        import torch

        return None if self.comm_dtype == "auto" else {"bf16": torch.bfloat16, "fp32": torch.float32}[self.comm_dtype]

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d["model"] = self.model.to_dict()
        return d

    @classmethod
    def from_dict(cls, d: dict) -> "TrainConfig":
        d = dict(d)
        model = d.pop("model", None)
        optim = d.pop("optim", None)
        data = d.pop("data", None)
        cfg = cls(**d)
        if isinstance(model, str):
            cfg.model = get_preset(model)
        elif isinstance(model, dict):
            cfg.model = ModelConfig.from_dict(model)
        if optim:
            cfg.optim = OptimConfig(**{**dataclasses.asdict(OptimConfig()), **optim})
            cfg.optim.betas = tuple(cfg.optim.betas)
        if data:
            cfg.data = DataConfig(**{**dataclasses.asdict(DataConfig()), **data})
        return cfg

    @classmethod
    def from_json(cls, path: str | Path) -> "TrainConfig":
        return cls.from_dict(json.loads(Path(path).read_text()))


def apply_overrides(cfg: TrainConfig, overrides: list[str]) -> TrainConfig:
    """Apply ``a.b.c=value`` overrides (value parsed as JSON when possible)."""
    for ov in overrides:
        key, _, raw = ov.partition("=")
        try:
            val = json.loads(raw)
        except json.JSONDecodeError:
            val = raw
        obj = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            obj = getattr(obj, p)
        if not hasattr(obj, parts[-1]):
            raise KeyError(f"unknown config key {key!r}")
        setattr(obj, parts[-1], tuple(val) if isinstance(val, list) else val)
    return cfg
