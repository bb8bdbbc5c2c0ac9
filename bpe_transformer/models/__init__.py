"""Model zoo: decoder-only Transformer LM and its building blocks."""

from . import functional
from .config import PRESETS, ModelConfig, get_preset
from .layers import (
    ActFFN,
    Embedding,
    Linear,
    MultiHeadSelfAttention,
    RMSNorm,
    RotaryPositionalEmbedding,
    SwiGLU,
    TransformerBlock,
)
from .generation import DecodeSession, KVCache
from .transformer import TransformerLM

__all__ = [
    "PRESETS",
    "ActFFN",
    "DecodeSession",
    "Embedding",
    "KVCache",
    "Linear",
    "ModelConfig",
    "MultiHeadSelfAttention",
    "RMSNorm",
    "RotaryPositionalEmbedding",
    "SwiGLU",
    "TransformerBlock",
    "TransformerLM",
    "functional",
    "get_preset",
]
