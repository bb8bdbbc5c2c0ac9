"""The reference's import path for its GELU kernel (``bpe_transformer/kernels/triton/gelu.py``).

Only the module path is kept, so ``from bpe_transformer.kernels.triton.gelu import gelu`` works for code written
against the reference; nothing here uses Triton -- the op is the gfx950 HIP kernel of ``ops/csrc/activations.hip``.
"""
