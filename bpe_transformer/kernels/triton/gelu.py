"""``gelu`` at the reference's module path (``/root/reference/bpe_transformer/kernels/triton/gelu.py:18-30``).

The reference launches a forward-only Triton kernel over 1 024-element blocks and asserts a contiguous CUDA input.
Here the same tanh-approximation GELU, ``0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))``, runs the hand-written
gfx950 HIP kernel (``ops/csrc/activations.hip``: 16 bytes per lane, overflow-safe tanh, with a backward) for GPU
tensors and the fp32 formula on the CPU.  No Triton is imported.
"""

from __future__ import annotations

from torch import Tensor

from ...ops.activations import gelu as _gelu

BLOCK_SIZE = 1024  # the reference's elements per program; kept as a module constant for API parity


def gelu(x: Tensor) -> Tensor:
    """tanh-GELU of ``x`` (any shape; fp32 / bf16 on the GPU through the HIP kernel)."""
    return _gelu(x)


__all__ = ["gelu", "BLOCK_SIZE"]
