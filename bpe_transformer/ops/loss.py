"""Cross-entropy ops (``csrc/cross_entropy.hip``).

``lm_head_cross_entropy`` is the LM head plus softmax-CE as one autograd node (the GEMMs are separate kernels:
hipBLASLt for the logits and the input gradient, the ping-pong kernel for the weight gradient; the CE is a
register-resident HIP kernel between them).  Two modes:

* ``"logits"`` (default, fastest measured): the logits buffer is written once
  by the hipBLASLt GEMM, read by the CE kernel which overwrites it IN PLACE with
  ``(softmax - onehot) / n``, and the backward is two GEMMs scaled by the
  incoming gradient (applied to the small GEMM outputs, never to the
  [tokens, vocab] buffer).  One [tokens, vocab] bf16 buffer lives from forward
  to backward (13.2 GB at GPT-2 B 128) instead of logits + probabilities +
  gradient.
* ``"streamed"``: the full logits are never materialised.  Token chunks of
  ``chunk`` rows run GEMM -> CE (in place) -> dh = dlogits W and
  dW += dlogits^T h inside the forward, through ONE reused [chunk, vocab]
  buffer; only dh ([tokens, d]) and an fp32 dW ([vocab, d]) are kept for the
  backward, which scales them by the incoming gradient.  Same GEMM FLOPs as
  "logits" (nothing is recomputed: the gradient of a mean CE needs only the
  row's own softmax, known once its chunk's logits exist), memory
  O(chunk * vocab).  Chunking over the vocabulary instead would need an
  online max / sum across vocab chunks and a second logits pass for the
  gradient -- 50 % more head FLOPs for the same memory bound.

Reference contract K13 (``tests/adapters.py:440-455``).
"""

from __future__ import annotations

import os

import torch
from torch import Tensor

from . import reference as F
from ._ext import ops

IGNORE_INDEX = -100


def default_lmhead_chunk() -> int:
    """Token-chunk size of the LM head + CE when the caller passes none: ``BPE_LMHEAD_CHUNK`` (0 = one GEMM and one
    CE pass over the whole buffer, the measured default: ``docs/performance.md``, knob A/B)."""
    return int(os.environ.get("BPE_LMHEAD_CHUNK", "0"))


def default_lmhead_mode() -> str:
    """``BPE_LMHEAD_MODE``: ``logits`` (default) or ``streamed`` (see the module docstring)."""
    m = os.environ.get("BPE_LMHEAD_MODE", "logits")
    if m not in ("logits", "streamed"):
        raise ValueError(f"BPE_LMHEAD_MODE must be 'logits' or 'streamed', got {m!r}")
    return m


STREAMED_DEFAULT_CHUNK = 16384

_HEAD_DX_TN = True  # module flag (tests compare the NN call)


def _head_dx(dlogits: Tensor, w: Tensor, scale: Tensor | None = None) -> Tensor:
    """dh = dlogits @ (scale * W) in hipBLASLt's TN layout through a transposed copy of W (``ops.transpose_bf16``,
    as the blocks' input gradients do: models/fused_block.py ``_dx_tn``): 7.24 vs 8.27 ms at GPT-2 B 128 with tuned
    solutions (profiles/bench/head_dx_layouts_b128.log), +0.65 % end to end.  ``scale`` (the loss's upstream
    gradient, a device scalar) is applied inside that copy -- no elementwise pass over dh."""
    if (_HEAD_DX_TN and w.dtype == torch.bfloat16 and dlogits.is_cuda and w.stride(1) == 1
            and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0):
        sc = None if scale is None else scale.detach().float().reshape(1).contiguous()
        return torch.matmul(dlogits, ops().transpose_bf16(w, sc).t())
    dh = torch.matmul(dlogits, w)
    return dh if scale is None else dh * scale.to(dh.dtype)


class _LMHeadCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: Tensor, w: Tensor, targets: Tensor, ignore_index: int, chunk: int):
        V = w.shape[0]
        # zero-row padded weight (flat buffer, optim/flat.py): aligned GEMM shapes and logits row stride; the
        # pad columns of the logits are exactly 0 and the CE kernel never touches them, so their "gradient"
        # stays 0 and contributes nothing to dh or dW
        wp = getattr(w, "_bpe_padded", None)
        if wp is None or wp.data_ptr() != w.data_ptr():
            wp = w
        nvalid = (targets != ignore_index).sum().clamp_min(1).to(torch.float32)
        M = h.shape[0]
        chunk = chunk if 0 < chunk < M else M
        if chunk == M:
            logits = torch.matmul(h, wp.t())  # hipBLASLt
            loss_rows, _ = ops().ce_fwd_bwd(logits[:, :V], targets, ignore_index, True, nvalid)
        else:
            # token chunks: each chunk's logits are still in the Infinity Cache when the CE kernel reads and
            # rewrites them (one HBM pass instead of three over the [tokens, vocab] buffer).  Every chunk divides
            # by the GLOBAL count of valid targets, so the chunked loss and gradient equal the one-pass ones; the
            # last chunk may be short.
            logits = h.new_empty(M, wp.shape[0])
            parts = []
            for c0 in range(0, M, chunk):
                c1 = min(M, c0 + chunk)
                torch.matmul(h[c0:c1], wp.t(), out=logits[c0:c1])
                parts.append(ops().ce_fwd_bwd(logits[c0:c1, :V], targets[c0:c1], ignore_index, True, nvalid)[0])
            loss_rows = torch.cat(parts)
        ctx.save_for_backward(h, wp, logits)
        ctx.w_param = w
        ctx.padded = wp is not w
        return loss_rows.sum() / nvalid

    @staticmethod
    def backward(ctx, g: Tensor):
        h, w, dlogits = ctx.saved_tensors
        # the upstream scale goes on the small operands, never on the logits -- and where the GEMMs read transposed
        # copies of them anyway (W^T for dh, h^T for dW's "ppt" route) it is applied inside those copies, so no
        # elementwise pass over the [T, d] tensors runs (two ~75 us kernels per GPT-2 B 128 step before)
        dh = _head_dx(dlogits, w, g)
        mg = getattr(ctx.w_param, "_bpe_padded_grad" if ctx.padded else "main_grad", None)
        if ctx.padded and mg is None:
            return dh, torch.matmul(dlogits.t(), h * g.to(h.dtype))[: ctx.w_param.shape[0]], None, None, None
        if mg is not None:
            # weight gradient accumulated in place into the flat gradient buffer (no temporary, no grad add)
            from .gemm import accumulate_weight_grad

            accumulate_weight_grad(mg, dlogits, h, x_scale=g)
            cb = getattr(ctx.w_param, "_bpe_grad_ready", None)
            if cb is not None:
                cb(ctx.w_param)
            return dh, None, None, None, None
        return dh, torch.matmul(dlogits.t(), h * g.to(h.dtype)), None, None, None


class _LMHeadCEStreamedFn(torch.autograd.Function):
    """The ``"streamed"`` mode: loss, dh and dW formed chunk by chunk in the forward (module docstring)."""

    @staticmethod
    def forward(ctx, h: Tensor, w: Tensor, targets: Tensor, ignore_index: int, chunk: int):
        from .gemm import accumulate_weight_grad

        V = w.shape[0]
        wp = getattr(w, "_bpe_padded", None)
        if wp is None or wp.data_ptr() != w.data_ptr():
            wp = w
        nvalid = (targets != ignore_index).sum().clamp_min(1).to(torch.float32)
        M = h.shape[0]
        chunk = min(chunk, M)
        buf = h.new_empty(chunk, wp.shape[0])
        dh = torch.empty_like(h)
        dw = torch.zeros(wp.shape, device=h.device, dtype=torch.float32)
        parts = []
        for c0 in range(0, M, chunk):
            c1 = min(M, c0 + chunk)
            lc = buf[: c1 - c0]
            torch.matmul(h[c0:c1], wp.t(), out=lc)
            # pad columns (zero weight rows) are exactly 0 and untouched by the CE kernel: no dh / dW contribution
            parts.append(ops().ce_fwd_bwd(lc[:, :V], targets[c0:c1], ignore_index, True, nvalid)[0])
            dh[c0:c1] = _head_dx(lc, wp)
            accumulate_weight_grad(dw, lc, h[c0:c1])
        ctx.save_for_backward(dh, dw)
        ctx.w_param = w
        return torch.cat(parts).sum() / nvalid

    @staticmethod
    def backward(ctx, g: Tensor):
        dh, dw = ctx.saved_tensors
        w = ctx.w_param
        dh = dh * g.to(dh.dtype)
        rows = w.shape[0]
        padded = getattr(w, "_bpe_padded", None) is not None and w._bpe_padded.data_ptr() == w.data_ptr()
        mg = getattr(w, "_bpe_padded_grad" if padded else "main_grad", None)
        if mg is not None:
            mg.add_((dw[: mg.shape[0]] * g.float()).to(mg.dtype))
            cb = getattr(w, "_bpe_grad_ready", None)
            if cb is not None:
                cb(w)
            return dh, None, None, None, None
        return dh, (dw[:rows] * g.float()).to(w.dtype), None, None, None


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits: Tensor, targets: Tensor, ignore_index: int):
        buf = logits.detach().reshape(-1, logits.shape[-1]).clone()
        loss_rows, _ = ops().ce_fwd_bwd(buf, targets, ignore_index, True)
        nvalid = (targets != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(buf)
        ctx.shape = logits.shape
        return loss_rows.sum() / nvalid

    @staticmethod
    def backward(ctx, g: Tensor):
        (buf,) = ctx.saved_tensors
        return (buf * g.to(buf.dtype)).view(ctx.shape), None, None


def cross_entropy(logits: Tensor, targets: Tensor, ignore_index: int = IGNORE_INDEX) -> Tensor:
    """Mean cross-entropy over all rows of ``logits[..., V]``."""
    t = targets.reshape(-1)
    if logits.is_cuda and logits.dtype in (torch.float32, torch.bfloat16):
        return _CrossEntropyFn.apply(logits, t.long().contiguous(), ignore_index)
    x = logits.reshape(-1, logits.shape[-1])
    valid = t != ignore_index
    if bool(valid.all()):
        return F.cross_entropy(x, t)
    return F.cross_entropy(x[valid], t[valid])


@torch.no_grad()
def _lm_head_ce_loss_only(h: Tensor, w: Tensor, targets: Tensor, ignore_index: int, chunk: int) -> Tensor:
    V = w.shape[0]
    wp = getattr(w, "_bpe_padded", None)
    if wp is None or wp.data_ptr() != w.data_ptr():
        wp = w
    M = h.shape[0]
    chunk = min(chunk, M)
    nvalid = (targets != ignore_index).sum().clamp_min(1).to(torch.float32)
    buf = h.new_empty(chunk, wp.shape[0])
    total = torch.zeros((), device=h.device, dtype=torch.float32)
    for c0 in range(0, M, chunk):
        c1 = min(M, c0 + chunk)
        lg = buf[: c1 - c0]
        torch.matmul(h[c0:c1], wp.t(), out=lg)
        total += ops().ce_fwd_bwd(lg[:, :V], targets[c0:c1], ignore_index, False, nvalid)[0].sum()
    return total / nvalid


def lm_head_cross_entropy(h: Tensor, weight: Tensor, targets: Tensor, ignore_index: int = IGNORE_INDEX,
                          chunk: int | None = None, mode: str | None = None) -> Tensor:
    """``cross_entropy(h @ weight.T, targets)`` without keeping separate logits/probs/grad buffers.

    h: ``[..., d]``, weight: ``[V, d]``, targets: ``[...]``.  ``mode``: ``"logits"`` or ``"streamed"`` (module
    docstring; None = :func:`default_lmhead_mode`).  ``chunk``: token-chunk rows (logits mode: 0 = one pass,
    None = :func:`default_lmhead_chunk`; streamed mode: the reused buffer's rows, None / 0 =
    ``STREAMED_DEFAULT_CHUNK``).
    """
    mode = mode or default_lmhead_mode()
    d = h.shape[-1]
    h2 = h.reshape(-1, d)
    t = targets.reshape(-1).long().contiguous()
    if h.is_cuda and h.dtype == torch.bfloat16 and not (
            torch.is_grad_enabled() and (h.requires_grad or weight.requires_grad)):
        # no backward will run (evaluation / validation loss): loss only, chunk by chunk through one reused
        # buffer -- neither the full logits of "logits" mode nor the dh / dW work of "streamed" mode
        return _lm_head_ce_loss_only(h2, weight, t, ignore_index, int(chunk or STREAMED_DEFAULT_CHUNK))
    if h.is_cuda and h.dtype == torch.bfloat16 and mode == "streamed":
        return _LMHeadCEStreamedFn.apply(h2, weight, t, ignore_index, int(chunk or STREAMED_DEFAULT_CHUNK))
    if chunk is None:
        chunk = default_lmhead_chunk()
    if h.is_cuda and h.dtype in (torch.float32, torch.bfloat16):
        return _LMHeadCEFn.apply(h2, weight, t, ignore_index, int(chunk))
    return cross_entropy(h2 @ weight.t(), t, ignore_index)
