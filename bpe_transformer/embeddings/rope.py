"""Rotary positional embedding (contract K8, ``tests/adapters.py:187-206``).

The module lives in ``models.layers``; on the GPU training path RoPE is fused
into the flash-attention Q/K loads (``ops/csrc/flash_attn_fwd.hip``) and the
standalone kernel is ``ops/csrc/rope.hip``.
"""

from ..models.layers import RotaryPositionalEmbedding
from ..ops.rope import apply_rope

__all__ = ["RotaryPositionalEmbedding", "apply_rope"]
