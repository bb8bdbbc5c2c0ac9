"""Oracle functional ops (re-exported from :mod:`bpe_transformer.ops.reference`)."""

from ..ops.reference import (  # noqa: F401
    apply_rope,
    causal_mask,
    cross_entropy,
    gelu_tanh,
    log_softmax,
    rmsnorm,
    rope_tables,
    scaled_dot_product_attention,
    silu,
    softmax,
)
