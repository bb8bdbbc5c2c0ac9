"""Rotary positional embedding (contract K8, ``tests/adapters.py:187-206``).

The module lives in ``models.layers``.  On the GPU training path RoPE is applied in
the epilogue of the QKV projection GEMM (``ops/csrc/gemm_pp.hip`` ``EPI_ROPE``; the
fp8 path: ``gemm_fp8_rope``), and the attention kernels read the pre-rotated Q / K;
the standalone in-place kernel is ``ops/csrc/rope.hip`` (``rope_qk_``, used where
the fused GEMM does not apply).
"""

from ..models.layers import RotaryPositionalEmbedding
from ..ops.rope import apply_rope

__all__ = ["RotaryPositionalEmbedding", "apply_rope"]
