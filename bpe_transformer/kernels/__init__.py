"""Standalone GPU kernels with the reference's module layout.

The reference ships one GPU kernel, a forward-only Triton tanh-GELU
(``bpe_transformer/kernels/triton/gelu.py:18-64``).  Here the same op is a
gfx950 HIP kernel (``ops/csrc/activations.hip``, vectorised 16 B per lane,
overflow-safe tanh) with a backward, exposed as :func:`gelu`.
"""

from .gelu import gelu

__all__ = ["gelu"]
