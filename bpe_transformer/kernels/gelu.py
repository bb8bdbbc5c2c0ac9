"""tanh-approximation GELU: ``0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3)))``.

Reference: ``bpe_transformer/kernels/triton/gelu.py:18-30`` (host wrapper, CUDA
and contiguous input required, forward only).  This version runs the HIP kernel
for GPU tensors (fp32/bf16, any layout -- non-contiguous inputs are copied),
supports autograd, and computes the fp32 oracle on the CPU.
"""

from __future__ import annotations

from torch import Tensor

from ..ops.activations import gelu as _gelu


def gelu(x: Tensor) -> Tensor:
    return _gelu(x)
