"""Adapter layer binding the reference's test contract to this framework.

The reference defines its Transformer capabilities only as the adapter
signatures of its ``tests/adapters.py``; every adapter here has
the same name and signature and calls into ``bpe_transformer``.  Tensors on
the CPU run the fp32 oracle path; tensors on the GPU run the HIP kernels.
"""

from __future__ import annotations

import os
from collections.abc import Iterable
from typing import IO, Any, BinaryIO

import numpy as np
import torch
from torch import Tensor

from bpe_transformer import ops
from bpe_transformer import train_bpe as _train_bpe
from bpe_transformer.data import get_batch
from bpe_transformer.models import (
    Embedding,
    Linear,
    MultiHeadSelfAttention,
    RMSNorm,
    RotaryPositionalEmbedding,
    SwiGLU,
    TransformerBlock,
    TransformerLM,
)
from bpe_transformer.optim import AdamW, clip_grad_norm_, get_lr_cosine_schedule
from bpe_transformer.tokenization.bpe_tokenizer import BPETokenizer
from bpe_transformer.utils import load_checkpoint, save_checkpoint


def _dev_dtype(t: Tensor):
    return dict(device=t.device, dtype=t.dtype)


def run_linear(d_in: int, d_out: int, weights: Tensor, in_features: Tensor) -> Tensor:
    m = Linear(d_in, d_out, **_dev_dtype(weights))
    m.load_state_dict({"weight": weights})
    return m(in_features)


def run_embedding(vocab_size: int, d_model: int, weights: Tensor, token_ids: Tensor) -> Tensor:
    m = Embedding(vocab_size, d_model, **_dev_dtype(weights))
    m.load_state_dict({"weight": weights})
    return m(token_ids)


def run_swiglu(d_model: int, d_ff: int, w1_weight: Tensor, w2_weight: Tensor, w3_weight: Tensor,
               in_features: Tensor) -> Tensor:
    m = SwiGLU(d_model, d_ff, **_dev_dtype(w1_weight))
    m.load_state_dict({"w1.weight": w1_weight, "w2.weight": w2_weight, "w3.weight": w3_weight})
    return m(in_features)


def run_scaled_dot_product_attention(Q: Tensor, K: Tensor, V: Tensor, mask: Tensor | None = None) -> Tensor:
    return ops.scaled_dot_product_attention(Q, K, V, mask)  # GPU tensors: csrc/masked_sdpa.hip


def _mha(d_model, num_heads, q, k, v, o, max_seq_len=None, theta=None):
    m = MultiHeadSelfAttention(d_model, num_heads, max_seq_len, theta, use_rope=theta is not None,
                               **_dev_dtype(q))
    m.load_state_dict({"q_proj.weight": q, "k_proj.weight": k, "v_proj.weight": v, "output_proj.weight": o},
                      strict=False)
    return m


def run_multihead_self_attention(d_model: int, num_heads: int, q_proj_weight: Tensor, k_proj_weight: Tensor,
                                 v_proj_weight: Tensor, o_proj_weight: Tensor, in_features: Tensor) -> Tensor:
    return _mha(d_model, num_heads, q_proj_weight, k_proj_weight, v_proj_weight, o_proj_weight)(in_features)


def run_multihead_self_attention_with_rope(d_model: int, num_heads: int, max_seq_len: int, theta: float,
                                           q_proj_weight: Tensor, k_proj_weight: Tensor, v_proj_weight: Tensor,
                                           o_proj_weight: Tensor, in_features: Tensor,
                                           token_positions: Tensor | None = None) -> Tensor:
    m = _mha(d_model, num_heads, q_proj_weight, k_proj_weight, v_proj_weight, o_proj_weight, max_seq_len, theta)
    return m(in_features, token_positions)


def run_rope(d_k: int, theta: float, max_seq_len: int, in_query_or_key: Tensor, token_positions: Tensor) -> Tensor:
    rope = RotaryPositionalEmbedding(theta, d_k, max_seq_len, device=in_query_or_key.device)
    return rope(in_query_or_key, token_positions)


def run_transformer_block(d_model: int, num_heads: int, d_ff: int, max_seq_len: int, theta: float,
                          weights: dict[str, Tensor], in_features: Tensor) -> Tensor:
    w0 = next(iter(weights.values()))
    blk = TransformerBlock(d_model, num_heads, d_ff, max_seq_len, theta, **_dev_dtype(w0))
    blk.load_state_dict(weights)
    return blk(in_features)


def run_transformer_lm(vocab_size: int, context_length: int, d_model: int, num_layers: int, num_heads: int,
                       d_ff: int, rope_theta: float, weights: dict[str, Tensor], in_indices: Tensor) -> Tensor:
    w0 = next(iter(weights.values()))
    lm = TransformerLM(vocab_size, context_length, d_model, num_layers, num_heads, d_ff, rope_theta,
                       **_dev_dtype(w0))
    lm.load_reference_state_dict(weights)
    return lm(in_indices)


def run_rmsnorm(d_model: int, eps: float, weights: Tensor, in_features: Tensor) -> Tensor:
    m = RMSNorm(d_model, eps, **_dev_dtype(weights))
    m.load_state_dict({"weight": weights})
    return m(in_features)


def run_silu(in_features: Tensor) -> Tensor:
    return ops.silu(in_features)


def run_get_batch(dataset: np.ndarray, batch_size: int, context_length: int, device: str
                  ) -> tuple[torch.Tensor, torch.Tensor]:
    return get_batch(dataset, batch_size, context_length, device)


def run_softmax(in_features: Tensor, dim: int) -> Tensor:
    return ops.softmax(in_features, dim)


def run_cross_entropy(inputs: Tensor, targets: Tensor) -> Tensor:
    return ops.cross_entropy(inputs, targets)


def run_gradient_clipping(parameters: Iterable[torch.nn.Parameter], max_l2_norm: float) -> None:
    clip_grad_norm_(list(parameters), max_l2_norm)


def get_adamw_cls() -> Any:
    return AdamW


def run_get_lr_cosine_schedule(it: int, max_learning_rate: float, min_learning_rate: float, warmup_iters: int,
                               cosine_cycle_iters: int):
    return get_lr_cosine_schedule(it, max_learning_rate, min_learning_rate, warmup_iters, cosine_cycle_iters)


def run_save_checkpoint(model: torch.nn.Module, optimizer: torch.optim.Optimizer, iteration: int,
                        out: str | os.PathLike | BinaryIO | IO[bytes]):
    save_checkpoint(model, optimizer, iteration, out)


def run_load_checkpoint(src: str | os.PathLike | BinaryIO | IO[bytes], model: torch.nn.Module,
                        optimizer: torch.optim.Optimizer) -> int:
    return load_checkpoint(src, model, optimizer)


def get_tokenizer(vocab: dict[int, bytes], merges: list[tuple[bytes, bytes]],
                  special_tokens: list[str] | None = None) -> Any:
    return BPETokenizer(vocab=vocab, merges=merges, special_tokens=special_tokens)


def run_train_bpe(input_path: str | os.PathLike, vocab_size: int, special_tokens: list[str], **kwargs
                  ) -> tuple[dict[int, bytes], list[tuple[bytes, bytes]]]:
    return _train_bpe(input_path, vocab_size, special_tokens, **kwargs)
