"""Whole-block forward/backward for the GPU training path (pre-norm, RoPE, SwiGLU, causal).

One ``autograd.Function`` per transformer block instead of ~10 autograd nodes:

forward (x = xr + xd: the previous block's residual and its not-yet-added FFN output)::

    x, h1 = add_rmsnorm(xr, xd; ln1)  HIP (the residual add fused into the norm)
    qkv = h1 @ [Wq;Wk;Wv]^T, RoPE     our persistent ping-pong GEMM with RoPE on Q / K in its epilogue (D = 64
                                      and 128; fp8: the same in the hand fp8 kernel, gemm_fp8_rope)
    o = flash_attn(qkv)               HIP (csrc/flash_attn_fwd_v4.hip)
    g1 = o @ Wo^T                     hipBLASLt
    xm, h2 = add_rmsnorm(x, g1; ln2)  HIP
    gu, a = h2 @ [W1;W3]^T, silu(g)*u our ping-pong GEMM with the gate in its epilogue (csrc/gemm_pp.hip,
                                      d_model <= 1024; else hipBLASLt + the HIP gate kernel)
    g2 = a @ W2^T                     hipBLASLt; the block returns (xm, g2), added by the next norm
    (fp8 with fp8 weight gradients: the two norms write h1 / h2 and the gate writes a only as e4m3 in both
    layouts, and the gate's backward writes its gradient only as e5m2 in both layouts: ops/fp8.py
    add_rmsnorm_cast_t, swiglu_fwd_cast_t / swiglu_bwd_cast_t; the W13 GEMM itself writes a's two e4m3 layouts
    when the shapes allow, ops/fp8.py matmul_swiglu)

backward: the mirror image, with
  * the SwiGLU backward fused into the epilogue of the dY @ W2 GEMM (our
    ping-pong MFMA kernel): the gate gradient da never goes to HBM;
  * weight gradients ACCUMULATED IN PLACE into the flat gradient buffer
    (``param.main_grad``, set by the training engine) -- no temporary dW, no
    AccumulateGrad add kernels -- with the dW GEMMs that are ready together
    grouped into one split-K launch each (W2 + [W1;W3] after the SwiGLU
    backward, Wo + [Wq;Wk;Wv] after the attention backward: ops/gemm.py
    ``accumulate_weight_grads``), else by the per-shape route of ops/gemm.py;
  * the fused [Wq;Wk;Wv] and [W1;W3] weights and their gradients as zero-copy
    views of the flat buffers when the parameters are adjacent there (no
    torch.cat / split);
  * both residual-gradient additions folded into the RMSNorm backward kernel;
  * a data-parallel "gradient ready" notification per parameter right after
    its gradient lands, so bucketed all-reduces start while the rest of the
    backward runs.

Everything runs on the current stream.  (Weight-gradient GEMMs on a side stream were measured and removed:
912 k vs 1 006 k tok/s at GPT-2 B 128, ``profiles/bench/ab_lmhead_chunk_dwstream_b128.log`` -- the chip is
already full, so the two streams only compete for the same CUs.)

Without ``main_grad`` (e.g. a plain module, tests) the same function returns
ordinary per-parameter gradients.
"""

from __future__ import annotations

import math
import os

import torch
from torch import Tensor

from ..ops._ext import ops as hip
from ..ops.attention import prerotate_default
from ..ops.fp8 import (add_rmsnorm_cast_t, grads_swiglu, matmul_swiglu, norm_cast_ok, rope_ok, swiglu_bwd_cast_t,
                       swiglu_bwd_gemm_ok, swiglu_cast_ok, swiglu_fwd_cast_t, swiglu_gemm_ok)
from ..ops import gemm as _gemm
from ..ops.gemm import accumulate_weight_grad


def _adjacent_view(ts: list[Tensor]) -> Tensor | None:
    """[t0; t1; ...] along dim 0 as a view if the tensors are consecutive in one storage."""
    t0 = ts[0]
    es = t0.element_size()
    base = t0.untyped_storage().data_ptr()
    for a, b in zip(ts, ts[1:]):
        if not (a.is_contiguous() and b.is_contiguous() and a.shape[1:] == b.shape[1:]
                and b.untyped_storage().data_ptr() == base  # same allocation, not just neighbours
                and a.data_ptr() + a.numel() * es == b.data_ptr()):
            return None
    rows = sum(t.shape[0] for t in ts)
    return t0.as_strided((rows, *t0.shape[1:]), t0.stride())


def _cat_weights(ts: list[Tensor]) -> Tensor:
    v = _adjacent_view([t.detach() for t in ts])
    return v if v is not None else torch.cat([t.detach() for t in ts], 0)


def _fuse_swiglu_bwd(dy: Tensor, w2: Tensor, gu: Tensor) -> bool:
    """The fused dX-GEMM + SwiGLU-backward kernel covers tokens and d_ff in multiples of 256, d_model of 64."""
    return (dy.shape[0] % 256 == 0 and w2.shape[1] % 256 == 0 and dy.shape[1] % 64 == 0
            and gu.is_contiguous() and dy.stride(1) == 1 and w2.stride(1) == 1)


_FUSE_SWIGLU_FWD = True  # module flag (tests compare the unfused path)
_FUSE_SWIGLU_FWD_MAX_D = int(os.environ.get("BPE_FUSE_SWIGLU_FWD_MAX_D", "0"))  # d_model cap override (A/B knob)


def _fuse_swiglu_fwd(x: Tensor, w13: Tensor) -> bool:
    """The W13 GEMM with a = silu(g) * u in its epilogue (csrc/gemm_pp.hip EPI_SWIGLU_FWD): tokens in multiples
    of 256, d_ff of 128, d_model of 64; d_model up to 1024 at any token count, wider at >= 65 536 tokens.  Below
    that the library GEMM's lead over the ping-pong kernel outgrew the saved gate pass at d 2048: Llama-1.1B -1.2 %
    at B 8 (profiles/bench/ab_llama_swiglu_fwd_fused.log) and, until round 6, -0.6-0.9 % at B 32
    (ab_llama_swiglu_fused_b32.log, ab_llama_swiglu_fwd_fused_r5.log).  With the L2-aware tile order (gemm_pp.hip
    tile_rc: the fused GEMM 2.46 -> 2.25 ms at Llama s2048 B 32) the fused form wins there, +0.2 % end to end
    (profiles/bench/ab_llama_swiglu_fwd_fused_r6.log).  GPT-2 (d 768): +0.7 % (ab_e2e_swiglu_fwd_fused_b128.log).
    ``BPE_FUSE_SWIGLU_FWD_MAX_D`` > 0 replaces the rule with a plain d_model cap for A/Bs."""
    d, t = x.shape[1], x.shape[0]
    wide_ok = d <= _FUSE_SWIGLU_FWD_MAX_D if _FUSE_SWIGLU_FWD_MAX_D > 0 else (d <= 1024 or t >= 65536)
    return (_FUSE_SWIGLU_FWD and x.dtype == torch.bfloat16 and t % 256 == 0 and d % 64 == 0 and wide_ok
            and w13.shape[0] % 256 == 0 and x.stride(1) == 1 and w13.stride(1) == 1)


_FUSE_QKV_ROPE = True  # module flag (tests and A/B runs compare the unfused path)
# fp8 weight-gradient path: SwiGLU forward / backward write their outputs only as fp8 in both layouts (one pass with
# the cast, csrc/fp8.hip swiglu_cast_fp8_t) instead of bf16 plus a cast pass (module flag for tests and A/B runs)
_FP8_SWIGLU_CAST = True
# ... and the two RMSNorms write the QKV / W13 projections' inputs only as e4m3 in both layouts (module flag)
_FP8_NORM_CAST = True
# ... and the fp8 QKV projection runs on the hand fp8 kernel with RoPE in its epilogue instead of hipBLASLt + rope_qk_
_FP8_QKV_ROPE = True
# the RMSNorm weight gradients added into their flat gradient slots by the column-sum kernel (module flag for A/B)
_NORM_DW_ACC = True


def _fuse_qkv_rope(x: Tensor, w: Tensor, S: int) -> bool:
    """The QKV projection with RoPE in its epilogue (csrc/gemm_pp.hip EPI_ROPE) instead of hipBLASLt plus the
    in-place ``rope_qk_`` pass: tokens and the QKV width in multiples of 256, d_model of 64."""
    return (_FUSE_QKV_ROPE and x.dtype == torch.bfloat16 and x.shape[0] % 256 == 0 and x.shape[0] % S == 0
            and x.shape[1] % 64 == 0 and w.shape[0] % 256 == 0 and x.stride(1) == 1 and w.stride(1) == 1
            and x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0)


def _dx_tn(w: Tensor) -> bool:
    """Run dX = dY . W as dY . (W^T)^T with W^T materialised (``ops.transpose_bf16``): hipBLASLt's TN layout
    (both operands contiguous along the reduction) beats the NN layout of the stored weight by 10-20 % at the
    GPT-2 B 128 shapes, measured with tuned solutions on random data (benchmarks/gemm_layouts.py,
    profiles/bench/gemm_layouts_b128.log: qkv 0.359 vs 0.407 ms, o 0.138 vs 0.176, w13 0.606 vs 0.689); the
    transpose is ~3-7 us per weight."""
    return (w.dtype == torch.bfloat16 and w.stride(1) == 1 and w.stride(0) % 8 == 0
            and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0)


def _notify(p: Tensor) -> None:
    cb = getattr(p, "_bpe_grad_ready", None)
    if cb is not None:
        cb(p)


class FusedBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xr, xd, ln1, wq, wk, wv, wo, ln2, w1, w3, w2, cos, sin, meta):
        B, S, H, Hkv, D, eps, use_rope = meta[:7]
        # fp8: (e4m3 Fp8State, first slot, e5m2 gradient Fp8State or None, first gradient slot, fp8 weight
        # gradients) or None
        fp8 = meta[7]
        train = meta[8]  # a backward will run (decided by the caller: grad mode is off inside forward)
        scale = 1.0 / math.sqrt(D)
        w_qkv = _cat_weights([wq, wk, wv])
        w_13 = _cat_weights([w1, w3])
        # fp8 weight gradients: the norms write h1 / h2 only as e4m3 in both layouts (they feed nothing else)
        norm8 = (fp8 is not None and fp8[2] is not None and train and len(fp8) > 4 and bool(fp8[4])
                 and _FP8_NORM_CAST and norm_cast_ok(xr))
        # block input x2 = xr + xd: the previous block's residual and its un-added FFN output (residual adds
        # are fused into the following RMSNorm instead of a copy-then-accumulate GEMM)
        h1q = h2q = None
        if norm8:
            x2, h1q, r1 = add_rmsnorm_cast_t(fp8[0], xr, xd, ln1, eps, fp8[1] + 0)
            h1 = None
        elif xd is None:
            x2 = xr
            h1, r1 = hip().rmsnorm_fwd(x2, ln1, eps)
        else:
            x2, h1, r1 = hip().add_rmsnorm_fwd(xr, xd, ln1, eps)
        w8s = None
        xt8s = None
        if fp8 is not None:
            st, s0 = fp8[0], fp8[1]  # slots s0..s0+3: activations, s0+4..s0+7: weights
            keep = fp8[2] is not None  # fp8 input-gradient GEMMs reuse the quantised weights
            # fp8 weight gradients: the activation cast also writes X^T (e4m3) for dW = dY^T X
            wg = keep and train and len(fp8) > 4 and bool(fp8[4])
            w8s = []
            xt8s = [] if wg else None

            def mm(x, w, i, xq=None, rope=None):
                if not keep:
                    return st.matmul(x, w, s0 + i, s0 + 4 + i, rope=rope)
                y, w8t, xt8 = st.matmul(x, w, s0 + i, s0 + 4 + i, keep_w8=True, keep_xt=wg, xq=xq, rope=rope)
                w8s.append(w8t)
                if wg:
                    xt8s.append(xt8)
                return y

        pre = use_rope and prerotate_default(D)
        rope8 = False
        if fp8 is not None:
            xin = h1 if h1 is not None else h1q[0]
            rope8 = pre and _FP8_QKV_ROPE and rope_ok(xin, w_qkv, S)
            qkv = mm(h1, w_qkv, 0, xq=h1q, rope=(cos, sin, S, D, (H + Hkv) * D) if rope8 else None)
        if fp8 is None and pre and _fuse_qkv_rope(h1, w_qkv, S):
            # RoPE on Q / K in the projection's epilogue (saved rotated for the backward)
            qkv = hip().gemm_qkv_rope(h1, w_qkv, cos, sin, S, D, (H + Hkv) * D)
        else:
            if fp8 is None:
                qkv = torch.matmul(h1, w_qkv.t())
            if pre and not rope8:  # RoPE once, in place on Q / K of the QKV activation (saved rotated for the backward)
                hip().rope_qk_(qkv, cos, sin, B, S, H, Hkv, D)
        q, k, v = qkv[:, : H * D], qkv[:, H * D : (H + Hkv) * D], qkv[:, (H + Hkv) * D :]
        # training: the forward kernel zeroes the backward's fp32 dQ accumulator in its epilogue (hidden under
        # its compute; the backward pre-pass then only reads O / dO).  Only the fused atomics backward has that
        # accumulator (D != 64), and only when a backward will run.
        dq_acc = (torch.empty(B * ((S + 63) // 64 * 64), H * D, device=q.device, dtype=torch.float32)
                  if train and hip().fa_bwd_needs_dq_acc(D) else None)
        o, lse = hip().fa_fwd(q, k, v, cos, sin, B, S, H, Hkv, D, True, use_rope, scale, pre, dq_acc)
        ctx.dq_acc = dq_acc
        g1 = mm(o, wo.detach(), 1) if fp8 is not None else torch.matmul(o, wo.t())
        if norm8:
            xm, h2q, r2 = add_rmsnorm_cast_t(fp8[0], x2, g1, ln2, eps, fp8[1] + 2)
            h2 = None
        else:
            xm, h2, r2 = hip().add_rmsnorm_fwd(x2, g1, ln2, eps)
        aq = None  # fp8: a already quantised (both layouts) by the fused W13 GEMM
        if fp8 is None and _fuse_swiglu_fwd(h2, w_13):
            gu, a = hip().gemm_swiglu_fwd(h2, w_13)  # the gate in the GEMM epilogue: no second pass over gu
        elif (fp8 is not None and xt8s is not None and _FP8_SWIGLU_CAST and h2q is not None
              and swiglu_gemm_ok(h2q[0], w_13)):
            # fp8 with weight gradients: W13 GEMM + gate + two-layout e4m3 cast of a in one kernel (the
            # bookkeeping of mm(): the e4m3 W^T for the input gradient, X^T for the weight gradient)
            gu, w8t13, xt813, aq = matmul_swiglu(st, h2q, w_13, s0 + 2, s0 + 6, s0 + 3)
            w8s.append(w8t13)
            xt8s.append(xt813)
            a = None
        else:
            gu = mm(h2, w_13, 2, xq=h2q) if fp8 is not None else torch.matmul(h2, w_13.t())
            a = None if xt8s is not None and _FP8_SWIGLU_CAST and swiglu_cast_ok(gu) else hip().swiglu_fwd(gu)
        if a is None:
            # fp8 weight gradients: a = silu(g) u is written only as the W2 GEMM's fp8 operand, in both layouts,
            # by one pass over gu (no bf16 a, no separate cast) -- or already by the fused W13 GEMM
            g2 = mm(None, w2.detach(), 3, xq=aq if aq is not None else swiglu_fwd_cast_t(fp8[0], gu, fp8[1] + 3))
        else:
            g2 = mm(a, w2.detach(), 3) if fp8 is not None else torch.matmul(a, w2.t())
        ctx.w8s = w8s if w8s else None
        ctx.xt8s = xt8s
        ctx.has_xd = xd is not None
        if xt8s is not None:  # h1, h2, a only fed the bf16 weight gradients: not kept
            h1 = h2 = a = None
        ctx.save_for_backward(x2, r1, h1, qkv, o, lse, xm, r2, h2, gu, a, cos, sin)
        ctx.params = (ln1, wq, wk, wv, wo, ln2, w1, w3, w2)
        ctx.meta = meta
        ctx.prerotated = pre
        return xm, g2  # block output = xm + g2, added by the consumer

    @staticmethod
    def backward(ctx, dxm_out, dg2):
        x2, r1, h1, qkv, o, lse, xm, r2, h2, gu, a, cos, sin = ctx.saved_tensors
        ln1, wq, wk, wv, wo, ln2, w1, w3, w2 = ctx.params
        B, S, H, Hkv, D, eps, use_rope = ctx.meta[:7]
        scale = 1.0 / math.sqrt(D)
        dy = dg2.contiguous()  # gradient of the FFN output g2
        dxm_out = dxm_out.contiguous()  # gradient reaching xm through the residual stream
        params = ctx.params
        main = all(hasattr(p, "main_grad") for p in params)
        grads: dict[int, Tensor] = {}

        def acc_weight(ps: list[Tensor], g_out: Tensor, x_in: Tensor) -> None:
            """dW = g_out^T x_in for the row-stacked weights ``ps``, accumulated into their flat gradient slices."""
            if main:
                view = _adjacent_view([p.main_grad for p in ps])
                if view is not None:
                    accumulate_weight_grad(view, g_out, x_in)
                else:
                    off = 0
                    for p in ps:
                        n = p.shape[0]
                        accumulate_weight_grad(p.main_grad, g_out[:, off : off + n], x_in)
                        off += n
                for p in ps:
                    _notify(p)
            else:
                dw = torch.matmul(g_out.t(), x_in)
                off = 0
                for p in ps:
                    n = p.shape[0]
                    grads[id(p)] = dw[off : off + n]
                    off += n

        def acc_weights(sets: list[tuple[list[Tensor], Tensor, Tensor]]) -> None:
            """:func:`acc_weight` for several projections whose gradients are ready together: one grouped split-K
            launch (ops/gemm.py ``accumulate_weight_grads``) when every stacked weight's gradient slots are adjacent
            in the flat buffer, else one launch each."""
            if main and _gemm._GROUP:
                views = [_adjacent_view([p.main_grad for p in ps]) for ps, _, _ in sets]
                if all(v is not None for v in views):
                    _gemm.accumulate_weight_grads([(v, g_out, x_in) for v, (_, g_out, x_in) in zip(views, sets)])
                    for ps, _, _ in sets:
                        for p in ps:
                            _notify(p)
                    return
            for ps, g_out, x_in in sets:
                acc_weight(ps, g_out, x_in)

        fp8 = ctx.meta[7]
        w8s = getattr(ctx, "w8s", None)
        xt8s = getattr(ctx, "xt8s", None)
        if getattr(ctx, "consumed", False):
            # the fp8 weight-gradient path frees its saved fp8 activations (and h1 / h2 / a were never kept), and the
            # fused attention backward consumes dq_acc: a second backward through the same graph has no operands
            raise RuntimeError("FusedBlockFn: backward ran twice through the same graph (retain_graph=True); the "
                               "fused block frees its saved activations in its first backward")
        ctx.consumed = xt8s is not None or getattr(ctx, "dq_acc", None) is not None
        ctx.xt8s = None

        def acc_dw(ps: list[Tensor], dw: Tensor) -> None:
            """Add a formed weight gradient (the fp8 weight-gradient GEMM's bf16 output) for the row-stacked ``ps``."""
            if main:
                view = _adjacent_view([p.main_grad for p in ps])
                if view is not None:
                    view.add_(dw)
                else:
                    off = 0
                    for p in ps:
                        n = p.shape[0]
                        p.main_grad.add_(dw[off : off + n])
                        off += n
                for p in ps:
                    _notify(p)
            else:
                off = 0
                for p in ps:
                    n = p.shape[0]
                    grads[id(p)] = dw[off : off + n]
                    off += n

        def dx(g_out: Tensor, ws: list[Tensor], i: int) -> Tensor:
            """Input gradient g_out @ W of projection i (0 qkv, 1 o, 2 w13, 3 w2): fp8 e5m2 x e4m3 when enabled;
            bf16 in hipBLASLt's TN layout through a transposed weight copy (:func:`_dx_tn`)."""
            if w8s is not None:
                from ..ops.fp8 import dgrad

                return dgrad(fp8[2], g_out, fp8[3] + i, w8s[i], fp8[0], fp8[1] + 4 + i)
            w = ws[0].detach() if len(ws) == 1 else _cat_weights(ws)
            if _dx_tn(w):
                return torch.matmul(g_out, hip().transpose_bf16(w).t())
            return torch.matmul(g_out, w)

        def proj(g_out: Tensor | None, ws: list[Tensor], i: int, x_in: Tensor | None, gq=None) -> Tensor:
            """Both gradients of projection i: returns dX = g_out @ W, accumulates dW = g_out^T x_in.  With fp8
            weight gradients both come from one e5m2 cast of g_out (ops/fp8.py ``grads``), or from ``gq`` = g_out
            already quantised in both layouts by its producer."""
            if xt8s is not None:
                from ..ops.fp8 import grads as fp8_grads

                # accumulated straight into the flat gradient buffer when the stacked weights are adjacent there
                view = _adjacent_view([p.main_grad for p in ws]) if main else None
                dxv, dw = fp8_grads(fp8[2], g_out, fp8[3] + i, w8s[i], fp8[0], fp8[1] + 4 + i, xt8s[i], fp8[0],
                                    fp8[1] + i, dw_out=view, gq=gq)
                if view is None:
                    acc_dw(ws, dw)
                else:
                    for p in ws:
                        _notify(p)
                return dxv
            acc_weight(ws, g_out, x_in)
            return dx(g_out, ws, i)

        # ---- FFN
        dgu_q = None
        if w8s is None and _fuse_swiglu_bwd(dy, w2, gu):
            # da = dy @ W2 with the SwiGLU backward in the GEMM epilogue (csrc/gemm_pp.hip): da never reaches HBM
            dgu = hip().gemm_swiglu_bwd(dy, w2.detach(), gu)
            # the W2 and [W1; W3] weight gradients, both ready now, in one grouped split-K launch
            acc_weights([([w2], dy, a), ([w1, w3], dgu, h2)])
            dh2 = dx(dgu, [w1, w3], 2)
        elif (xt8s is not None and _FP8_SWIGLU_CAST and swiglu_cast_ok(gu)
              and swiglu_bwd_gemm_ok(dy, w8s[3], gu)):
            # fp8 weight gradients: one e5m2 cast of dy feeds W2's weight gradient and the hand kernel whose
            # epilogue turns da (never stored) into [dg | du] in e5m2, both layouts (the W13 projection's operands)
            view = _adjacent_view([w2.main_grad]) if main else None
            dgu_q, dw2 = grads_swiglu(fp8[2], dy, fp8[3] + 3, w8s[3], fp8[0], fp8[1] + 4 + 3, xt8s[3], fp8[0],
                                      fp8[1] + 3, view, gu, fp8[3] + 2)
            if view is None:
                acc_dw([w2], dw2)
            else:
                _notify(w2)
            dgu = None
            dh2 = proj(dgu, [w1, w3], 2, h2, gq=dgu_q)
        else:
            da = proj(dy, [w2], 3, a)
            if xt8s is not None and _FP8_SWIGLU_CAST and swiglu_cast_ok(gu):
                # the gate gradient straight to e5m2 in both layouts (the W13 projection's operands): no bf16 dgu
                dgu = None
                dgu_q = swiglu_bwd_cast_t(fp8[2], da, gu, fp8[3] + 2)
            else:
                dgu = hip().swiglu_bwd(da, gu)
            dh2 = proj(dgu, [w1, w3], 2, h2, gq=dgu_q)
        # with flat gradient slots the norm weights' gradients are added there by the column-sum kernel itself
        nacc = main and _NORM_DW_ACC
        dxm, dln2 = hip().rmsnorm_bwd(dh2, xm, ln2.detach(), r2, dxm_out, ln2.main_grad if nacc else None)
        # ---- attention
        # bf16 weight gradients: Wo's waits for the attention backward, so that it runs in one grouped launch with
        # [Wq; Wk; Wv]'s (dxm stays alive until the ln1 backward anyway)
        group_attn = xt8s is None and main and _gemm._GROUP
        do = dx(dxm, [wo], 1) if group_attn else proj(dxm, [wo], 1, o)
        q, k, v = qkv[:, : H * D], qkv[:, H * D : (H + Hkv) * D], qkv[:, (H + Hkv) * D :]
        dqkv = hip().fa_bwd(do, q, k, v, o, lse, cos, sin, B, S, H, Hkv, D, True, use_rope, scale, ctx.prerotated,
                            ctx.dq_acc)
        ctx.dq_acc = None
        if group_attn:
            acc_weights([([wo], dxm, o), ([wq, wk, wv], dqkv, h1)])
            dh1 = dx(dqkv, [wq, wk, wv], 0)
        else:
            dh1 = proj(dqkv, [wq, wk, wv], 0, h1)
        dx2, dln1 = hip().rmsnorm_bwd(dh1, x2, ln1.detach(), r1, dxm, ln1.main_grad if nacc else None)
        dxd = dx2 if ctx.has_xd else None
        if main:
            if not nacc:
                ln2.main_grad.add_(dln2)
                ln1.main_grad.add_(dln1)
            _notify(ln2)
            _notify(ln1)
            return (dx2, dxd) + (None,) * 12
        grads[id(ln1)] = dln1
        grads[id(ln2)] = dln2
        return (dx2, dxd, grads[id(ln1)], grads[id(wq)], grads[id(wk)], grads[id(wv)], grads[id(wo)], grads[id(ln2)],
                grads[id(w1)], grads[id(w3)], grads[id(w2)], None, None, None)


class AddRMSNormFn(torch.autograd.Function):
    """RMSNorm(xr + xd) with the residual add fused (the model's final norm after the last fused block)."""

    @staticmethod
    def forward(ctx, xr, xd, w, eps):
        s_, y, r = hip().add_rmsnorm_fwd(xr, xd, w, eps)
        ctx.save_for_backward(s_, w, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        s_, w, r = ctx.saved_tensors
        dx, dw = hip().rmsnorm_bwd(dy.contiguous(), s_, w.detach(), r, None)
        return dx, dx, dw.to(w.dtype), None


_EMPTY: dict = {}


def fused_block_pair(block, xr: Tensor, xd: Tensor | None, B: int, S: int) -> tuple[Tensor, Tensor]:
    """Run ``block`` on input ``xr + xd`` ([B*S, d] each; xd may be None); returns (residual, delta) whose sum
    is the block output -- the next block (or the final norm) adds them inside its RMSNorm."""
    attn, ffn = block.attn, block.ffn
    if attn.rope is not None:
        cos, sin, use_rope = attn.rope.cos, attn.rope.sin, True
    else:
        key = xr.device
        if key not in _EMPTY:
            _EMPTY[key] = torch.empty(0, 0, device=key, dtype=torch.float32)
        cos = sin = _EMPTY[key]
        use_rope = False
    train = torch.is_grad_enabled() and (xr.requires_grad or any(p.requires_grad for p in block.parameters()))
    meta = (B, S, attn.num_heads, attn.num_kv_heads, attn.d_k, block.ln1.eps, use_rope, getattr(block, "fp8", None),
            train)
    return FusedBlockFn.apply(xr, xd, block.ln1.weight, attn.q_proj.weight, attn.k_proj.weight,
                              attn.v_proj.weight, attn.output_proj.weight, block.ln2.weight, ffn.w1.weight,
                              ffn.w3.weight, ffn.w2.weight, cos, sin, meta)


def fused_block_forward(block, x: Tensor) -> Tensor:
    """Run one ``block`` (a TransformerBlock) through :class:`FusedBlockFn`; x: [B, S, d] bf16 on the GPU."""
    B, S, d = x.shape
    xm, g2 = fused_block_pair(block, x.reshape(B * S, d).contiguous(), None, B, S)
    return (xm + g2).view(B, S, d)


def fused_stack_forward(layers, ln_final, x: Tensor, fence=None) -> Tensor:
    """All blocks + the final RMSNorm with every residual add fused into the following norm.  ``fence``
    (optional callable(module)) runs before each module's weights are read (sharded DP weight all-gathers)."""
    B, S, d = x.shape
    xr, xd = x.reshape(B * S, d).contiguous(), None
    for layer in layers:
        if fence is not None:
            fence(layer)
        xr, xd = fused_block_pair(layer, xr, xd, B, S)
    if fence is not None:
        fence(ln_final)
    return AddRMSNormFn.apply(xr, xd, ln_final.weight, ln_final.eps).view(B, S, d)
