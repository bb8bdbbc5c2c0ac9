"""gfx950 (MI355X) HIP kernel ops.

Every op runs its hand-written HIP kernel when its inputs live on the GPU and
the plain-PyTorch oracle (``models.functional``) on the CPU.  The device path
never silently falls back: if ``_bpe_hip.so`` is missing on a GPU machine the
first op raises (see ``ops._ext``).  GEMMs stay on hipBLASLt via
``torch.matmul``/``addmm`` (plain library GEMMs); every non-GEMM op of the
training step is here.
"""

from ._ext import is_built, library_path, load
from .activations import gelu, silu, swiglu_gate
from .attention import attention_qkv_reference, flash_attention_qkv, flash_supported, scaled_dot_product_attention
from .decode import decode_attention, kv_append
from .embedding import embedding
from .loss import IGNORE_INDEX, cross_entropy, lm_head_cross_entropy
from .norm import rmsnorm
from .optim import clip_grad_norm_, fused_adamw_step, grad_norm
from .rope import apply_rope
from .softmax import softmax

__all__ = [
    "IGNORE_INDEX",
    "apply_rope",
    "attention_qkv_reference",
    "clip_grad_norm_",
    "cross_entropy",
    "decode_attention",
    "embedding",
    "flash_attention_qkv",
    "flash_supported",
    "fused_adamw_step",
    "gelu",
    "grad_norm",
    "is_built",
    "kv_append",
    "library_path",
    "lm_head_cross_entropy",
    "load",
    "rmsnorm",
    "scaled_dot_product_attention",
    "silu",
    "softmax",
    "swiglu_gate",
]
