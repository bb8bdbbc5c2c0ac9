"""FP8 (OCP e4m3fn) forward projections with delayed per-tensor scaling.

Recipe (BASELINE.json "Llama-style 1.1B fp8 MFMA path"):
  * the four projection GEMMs of every block run as fp8 x fp8 -> bf16 on the
    MFMA fp8 units.  Which kernel serves which GEMM at the bench config
    (Llama-1.1B, s4096 B16 = 65 536 tokens):
      - the QKV forward: the hand-written ping-pong kernel with
        ``v_mfma_scale_f32_16x16x128_f8f6f4`` (``csrc/gemm_pp.hip``, F8; per-tensor
        inverse scales applied in its epilogue, read from the device) with RoPE
        in its epilogue (``gemm_fp8_rope``, :func:`rope_ok`);
      - every weight gradient: the hand kernel's split-K form
        (:func:`wgrad_acc`, ``gemm_fp8_acc``), 2.29-2.64 vs the library's
        1.65-2.09 PF/s (``profiles/bench/fp8_wgrad_r4.log``);
      - the W13 forward with weight gradients on: the hand kernel with the
        SwiGLU gate and its two-layout e4m3 cast in the epilogue
        (:func:`matmul_swiglu`; round 6);
      - the O / W2 forward (and W13 without fused casts) and every input
        gradient: hipBLASLt's ``torch._scaled_mm``, which leads the hand kernel
        by 3-12 % at these shapes (``profiles/bench/fp8_gemm_orders_r6.log``).  The route
        table ``ops/tuning/fp8_routes.json`` sends only its listed shapes (two
        16 384-token ones) to the hand kernel; ``BPE_FP8_GEMM=hip`` / ``lib`` force
        one path for all of :func:`mm_fp8`;
  * activations and weights are quantised by ``csrc/fp8.hip`` with a scale
    derived from an amax history (delayed scaling, powers of two); the cast
    pass also records this step's amax, and one launch per step refreshes all
    scales -- the host never reads a scale;
  * input-gradient GEMMs (dX = dY . W) optionally run in fp8 too: dY is
    quantised to e5m2 (wider range, the usual gradient format) with its own
    delayed scales, W reuses the forward's e4m3 copy (transposed once);
  * weight-gradient GEMMs (dW = dY^T . X) optionally as well (``wgrad``):
    they reduce over tokens, so the forward's activation cast also writes
    X^T (e4m3, [K, tokens], saved for the backward instead of nothing extra
    on the bf16 side) and the backward's one gradient cast writes dY and dY^T
    (e5m2) together (``cast_t``: both layouts in one pass, csrc/fp8.hip);
    master weights and optimizer state stay fp32.
"""

from __future__ import annotations

import json
import os

import torch
from torch import Tensor

from ._ext import ops

FP8 = torch.float8_e4m3fn
BF8 = torch.float8_e5m2
_FMT = {"e4m3": (FP8, 0), "e5m2": (BF8, 1)}
# BPE_FP8_GEMM: "routes" (default) = the HIP kernel for the shapes listed in ops/tuning/fp8_routes.json (where it
# measured faster than hipBLASLt), hipBLASLt elsewhere; "hip" = the HIP kernel wherever it applies; "lib" =
# hipBLASLt everywhere
_MODE = os.environ.get("BPE_FP8_GEMM", "routes")
if _MODE not in ("routes", "hip", "lib"):
    raise ValueError(f"BPE_FP8_GEMM must be routes, hip or lib, got {_MODE!r}")


def _load_routes() -> set[tuple[int, int, int, str]]:
    path = os.path.join(os.path.dirname(__file__), "tuning", "fp8_routes.json")
    try:
        with open(path) as f:
            table = json.load(f)
    except FileNotFoundError:
        return set()
    out = set()
    for key, route in table.get("routes", {}).items():
        m, n, k, fmt = key.split(",")
        if route == "hip":
            out.add((int(m), int(n), int(k), fmt))
    return out


_HIP_ROUTES = _load_routes()


def _use_hip(M: int, N: int, K: int, a_dtype) -> bool:
    if _MODE == "lib":
        return False
    if _MODE == "hip":
        return True
    return (M, N, K, "e5m2" if a_dtype == torch.float8_e5m2 else "e4m3") in _HIP_ROUTES


def mm_fp8(a8: Tensor, b8: Tensor, sa: Tensor, sb: Tensor) -> Tensor:
    """``(a8 @ b8.T) * sa * sb`` in bf16; a8 [M, K] e4m3 / e5m2, b8 [N, K] e4m3, sa / sb fp32 device scalars.

    The HIP fp8 MFMA kernel (``gemm_pp.hip``, F8) for the routed shapes (``BPE_FP8_GEMM``, above) when the shape is
    256 x 256 x 128-aligned, else hipBLASLt."""
    M, K = a8.shape
    N = b8.shape[0]
    # the hand kernel has no split-K: a weight-gradient shape (few output tiles, K = all tokens) would leave most
    # CUs idle, so those go to the library even when BPE_FP8_GEMM=hip
    few_tiles = (M // 256) * (N // 256) < 128 and K > 4 * max(M, N)
    if (not few_tiles and M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and _use_hip(M, N, K, a8.dtype)
            and a8.stride(1) == 1
            and b8.stride(1) == 1 and a8.stride(0) % 16 == 0 and b8.stride(0) % 16 == 0 and b8.dtype == FP8):
        return ops().gemm_fp8(a8, b8, sa.reshape(1), sb.reshape(1))
    return torch._scaled_mm(a8, b8.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)


class Fp8State:
    """Scaling state for ``n_slots`` quantised tensors of one format (device-resident)."""

    def __init__(self, n_slots: int, device, history: int = 16, margin: float = 1.0, fmt: str = "e4m3"):
        self.dtype, self.fmt_code = _FMT[fmt]
        self.fmt = fmt
        self.n = n_slots
        self.amax = torch.zeros(n_slots, dtype=torch.int32, device=device)
        self.hist = torch.zeros(n_slots, history, dtype=torch.float32, device=device)
        self.scale = torch.ones(n_slots, dtype=torch.float32, device=device)
        self.inv_scale = torch.ones(n_slots, dtype=torch.float32, device=device)
        self.margin = margin
        self.pos = 0
        # diagnostic (benchmarks/fp8_spike_probe.py): when a list, update() appends a [2, n] device tensor per step --
        # the step's amax per slot and the scale its casts used.  amax * scale / FMAX > 1 means values saturated.
        self.trace: list | None = None

    def cast(self, x: Tensor, slot: int) -> Tensor:
        out = torch.empty(x.shape, dtype=self.dtype, device=x.device)
        ops().cast_fp8(x.contiguous(), self.scale[slot : slot + 1], out, self.amax[slot : slot + 1])
        return out

    def update(self) -> None:
        """Fold this step's amaxes into the history and recompute every scale (one launch)."""
        if self.trace is not None:
            self.trace.append(torch.stack([self.amax.view(torch.float32).clone(), self.scale.clone()]))
        ops().update_scales(self.amax, self.hist, self.scale, self.inv_scale, self.pos, self.margin, self.fmt_code)
        self.pos += 1

    def state_dict(self) -> dict:
        """Scale state for checkpoints (amax history, current scales, ring position)."""
        return {"hist": self.hist.clone(), "scale": self.scale.clone(), "inv_scale": self.inv_scale.clone(),
                "pos": self.pos, "margin": self.margin}

    def load_state_dict(self, sd: dict) -> None:
        if sd["hist"].shape != self.hist.shape:
            raise ValueError(f"fp8 state shape {tuple(sd['hist'].shape)} != {tuple(self.hist.shape)}")
        self.hist.copy_(sd["hist"])
        self.scale.copy_(sd["scale"])
        self.inv_scale.copy_(sd["inv_scale"])
        self.amax.zero_()
        self.pos = int(sd["pos"])
        self.margin = float(sd["margin"])

    def cast_t(self, w: Tensor, slot: int) -> tuple[Tensor, Tensor]:
        """Two-layout cast of a bf16 [N, K] matrix (N, K multiples of 64): (w8 [N, K], w8t [K, N]) in this state's
        format, one pass (csrc/fp8.hip cast_fp8_t)."""
        w = w.contiguous()
        w8 = torch.empty(w.shape, dtype=self.dtype, device=w.device)
        w8t = torch.empty(w.shape[1], w.shape[0], dtype=self.dtype, device=w.device)
        ops().cast_fp8_t(w, self.scale[slot : slot + 1], w8, w8t, self.amax[slot : slot + 1])
        return w8, w8t

    def matmul(self, x: Tensor | None, w: Tensor, x_slot: int, w_slot: int, keep_w8: bool = False,
               keep_xt: bool = False, xq: tuple[Tensor, Tensor] | None = None, rope: tuple | None = None):
        """``x @ w.T`` in fp8 with bf16 output; x: [M, K] bf16, w: [N, K] bf16.  Without flags returns y.  With
        ``keep_w8`` / ``keep_xt`` returns ``(y, w8t, xt8)``: the quantised weight in the [K, N] layout the
        input-gradient GEMM needs and the quantised activation in the [K, M] layout of the weight-gradient GEMM
        (each written by the same cast pass as the forward operand; None when not asked for).  ``xq`` = (x8, xt8):
        x already quantised in both layouts by its producer in slot ``x_slot`` (``swiglu_fwd_cast_t``); x is then
        not read.  ``rope`` = (cos, sin, S, D, rot_cols): the QKV projection with RoPE on its first ``rot_cols`` output
        columns in the hand fp8 kernel's epilogue (the caller checks :func:`rope_ok`)."""
        xt8 = None
        if xq is not None:
            x8, xt8 = xq
        elif keep_xt:
            x8, xt8 = self.cast_t(x, x_slot) if _t_ok(x) else (self.cast(x, x_slot), None)
            if xt8 is None:
                xt8 = x8.t().contiguous()
        else:
            x8 = self.cast(x, x_slot)
        w8t = None
        if keep_w8 and _t_ok(w):
            w8, w8t = self.cast_t(w, w_slot)
        else:
            w8 = self.cast(w, w_slot)
            if keep_w8:
                w8t = w8.t().contiguous()
        if rope is not None:
            c, s, S, D, rot = rope
            y = ops().gemm_fp8_rope(x8, w8, self.inv_scale[x_slot : x_slot + 1], self.inv_scale[w_slot : w_slot + 1],
                                    c, s, S, D, rot)
        else:
            y = mm_fp8(x8, w8, self.inv_scale[x_slot], self.inv_scale[w_slot])
        if not keep_w8 and not keep_xt:
            return y
        return y, w8t, xt8


def rope_ok(x: Tensor, w: Tensor, S: int) -> bool:
    """Shapes the fp8 QKV GEMM with the RoPE epilogue takes: tokens and QKV width multiples of 256, d_model of 128,
    whole sequences."""
    return (x.shape[0] % 256 == 0 and w.shape[0] % 256 == 0 and x.shape[1] % 128 == 0 and x.shape[0] % S == 0
            and _MODE != "lib")


def _t_ok(t: Tensor) -> bool:
    """A bf16 matrix the two-layout cast takes (contiguous rows and columns in multiples of 64)."""
    return t.dtype == torch.bfloat16 and t.dim() == 2 and t.shape[0] % 64 == 0 and t.shape[1] % 64 == 0


def dgrad(g_state: Fp8State, g: Tensor, g_slot: int, w8t: Tensor, w_state: Fp8State, w_slot: int) -> Tensor:
    """``g @ W`` with g: [M, N] bf16 quantised to e5m2 (slot ``g_slot`` of ``g_state``) and W the forward's e4m3
    copy in the [K, N] layout ``w8t`` (its scale in slot ``w_slot`` of ``w_state``): both operands contiguous
    along the reduction (N), the layout of the fp8 kernel and of the library."""
    g8 = g_state.cast(g.contiguous(), g_slot)
    return mm_fp8(g8, w8t, g_state.inv_scale[g_slot], w_state.inv_scale[w_slot])


_WGRAD_HIP = True  # fp8 weight gradients on the hand kernel's split-K form (True) or hipBLASLt (module flag)


def wgrad_acc(g8t: Tensor, xt8: Tensor, sg: Tensor, sx: Tensor, out: Tensor) -> None:
    """``out += (g8t @ xt8.T) * sg * sx``: the fp8 weight gradient (g8t [N, tokens] e5m2, xt8 [K, tokens] e4m3)
    accumulated into a bf16 / fp32 gradient view [N, K].  The hand kernel's split-K form (fp32 partials and an
    ordered reduce with beta = 1 straight into ``out``) when ``_WGRAD_HIP`` and the shape is tile-aligned, else
    hipBLASLt's ``_scaled_mm`` and an add."""
    N, T = g8t.shape
    K = xt8.shape[0]
    if (_WGRAD_HIP and N % 256 == 0 and K % 256 == 0 and T % 128 == 0 and out.stride(1) == 1
            and g8t.stride(0) % 16 == 0 and xt8.stride(0) % 16 == 0):
        from .gemm import choose_splits_pp

        ops().gemm_fp8_acc(g8t, xt8, sg.reshape(1), sx.reshape(1), out, 1.0, choose_splits_pp(N, K, T // 2))
        return
    out.add_(torch._scaled_mm(g8t, xt8.t(), scale_a=sg, scale_b=sx, out_dtype=torch.bfloat16))


def grads(g_state: Fp8State, g: Tensor | None, g_slot: int, w8t: Tensor, w_state: Fp8State, w_slot: int,
          xt8: Tensor | None = None, x_state: Fp8State | None = None, x_slot: int = 0, dw_out: Tensor | None = None,
          gq: tuple[Tensor, Tensor] | None = None):
    """Input gradient ``g @ W`` and, with ``xt8``, weight gradient ``g^T @ X`` of one projection from ONE e5m2 cast
    of g: (dX, dW or None).  dW = g8t [N, tokens] x xt8 [K, tokens] -> [N, K], both operands contiguous along the
    token reduction; its scale is g's inverse scale times X's (slot ``x_slot`` of ``x_state``).  With ``dw_out``
    the weight gradient is accumulated into it (:func:`wgrad_acc`) and None is returned in its place.  ``gq`` =
    (g8, g8t): g already quantised in both layouts in slot ``g_slot`` by its producer (``swiglu_bwd_cast_t``)."""
    if xt8 is None:
        return dgrad(g_state, g, g_slot, w8t, w_state, w_slot), None
    if gq is not None:
        g8, g8t = gq
    else:
        g = g.contiguous()
        if _t_ok(g):
            g8, g8t = g_state.cast_t(g, g_slot)
        else:
            g8 = g_state.cast(g, g_slot)
            g8t = g8.t().contiguous()
    gi = g_state.inv_scale[g_slot]
    dx = mm_fp8(g8, w8t, gi, w_state.inv_scale[w_slot])
    if dw_out is not None:
        wgrad_acc(g8t, xt8, gi, x_state.inv_scale[x_slot], dw_out)
        return dx, None
    dw = mm_fp8(g8t, xt8, gi, x_state.inv_scale[x_slot])
    return dx, dw


def swiglu_cast_ok(gu: Tensor) -> bool:
    """gu = [g | u] that the fused SwiGLU + two-layout cast takes: bf16, contiguous, tokens and F multiples of 64."""
    return (gu.dtype == torch.bfloat16 and gu.dim() == 2 and gu.is_contiguous() and gu.shape[0] % 64 == 0
            and gu.shape[1] % 128 == 0)


def swiglu_fwd_cast_t(state: Fp8State, gu: Tensor, slot: int) -> tuple[Tensor, Tensor]:
    """a = silu(g) * u of gu = [g | u] ([M, 2F] bf16), written only in fp8 (this state's format, e4m3) in both layouts
    (a8 [M, F], a8t [F, M]; slot ``slot``): one pass instead of ``swiglu_fwd`` plus ``cast_t`` (csrc/fp8.hip)."""
    M, F = gu.shape[0], gu.shape[1] // 2
    a8 = torch.empty(M, F, dtype=state.dtype, device=gu.device)
    a8t = torch.empty(F, M, dtype=state.dtype, device=gu.device)
    ops().swiglu_cast_fp8_t(gu, None, state.scale[slot : slot + 1], a8, a8t, state.amax[slot : slot + 1])
    return a8, a8t


# BPE_FP8_SWIGLU_GEMM=0: the fp8 W13 GEMM (routed, hipBLASLt at the bench shapes) then swiglu_fwd_cast_t, instead
# of the hand kernel with the gate and its two-layout cast in the epilogue (swiglu_gemm_ok / matmul_swiglu)
_SWIGLU_GEMM = os.environ.get("BPE_FP8_SWIGLU_GEMM", "1") == "1"
# BPE_FP8_SWIGLU_BWD_GEMM=1: the W2 input gradient with the SwiGLU backward + e5m2 cast fused (swiglu_bwd_gemm_ok).
# Off by default: bitwise right but 1.89 vs 1.34 ms per Llama layer against hipBLASLt + swiglu_bwd_cast_t (its
# epilogue moves 512 KiB per tile -- g / u in, dg / du out in two layouts -- behind a 16-K-tile main loop, with
# register spills), fp8 step -3.6 % (profiles/bench/fp8_swiglu_gemm_r6.log)
_SWIGLU_BWD_GEMM = os.environ.get("BPE_FP8_SWIGLU_BWD_GEMM", "0") == "1"


def swiglu_gemm_ok(x8: Tensor, w13: Tensor) -> bool:
    """Shapes the fused fp8 W13 + SwiGLU + two-layout cast kernel takes: tokens a multiple of 256, d_ff of 128,
    d_model of 128, 32-bit operand offsets; never under ``BPE_FP8_GEMM=lib``."""
    M, K = x8.shape
    F2 = w13.shape[0]
    return (_SWIGLU_GEMM and _MODE != "lib" and x8.dtype == FP8 and x8.is_contiguous() and M % 256 == 0
            and F2 % 256 == 0 and K % 128 == 0 and K * 256 < 2**32 and F2 * K < 2**32)


def matmul_swiglu(state: Fp8State, xq: tuple[Tensor, Tensor], w13: Tensor, x_slot: int, w_slot: int, a_slot: int):
    """The fp8 W13 projection with the SwiGLU gate fused: ``gu = x8 @ w13_8.T`` (bf16, kept for the backward) and
    ``a = silu(g) * u`` written only in e4m3, both layouts, slot ``a_slot`` (csrc/gemm_pp.hip EPI_SWIGLU_FWD8) --
    the values of :meth:`Fp8State.matmul` + :func:`swiglu_fwd_cast_t` on the hand kernel, without the pass over gu.
    ``xq`` = (x8, xt8) from the producer (the fused norm cast).  Returns ``(gu, w8t, xt8, (a8, a8t))``."""
    x8, xt8 = xq
    if _t_ok(w13):
        w8, w8t = state.cast_t(w13, w_slot)
    else:
        w8 = state.cast(w13, w_slot)
        w8t = w8.t().contiguous()
    M, F = x8.shape[0], w13.shape[0] // 2
    a8 = torch.empty(M, F, dtype=state.dtype, device=x8.device)
    a8t = torch.empty(F, M, dtype=state.dtype, device=x8.device)
    gu = ops().gemm_fp8_swiglu(x8, w8.contiguous(), state.inv_scale[x_slot : x_slot + 1],
                               state.inv_scale[w_slot : w_slot + 1], state.scale[a_slot : a_slot + 1], a8, a8t,
                               state.amax[a_slot : a_slot + 1])
    return gu, w8t, xt8, (a8, a8t)


def swiglu_bwd_gemm_ok(g: Tensor, w8t: Tensor, gu: Tensor) -> bool:
    """Shapes the fused fp8 W2 input-gradient + SwiGLU backward + two-layout e5m2 cast kernel takes: tokens and d_ff
    multiples of 256, d_model of 128, 32-bit operand offsets, bf16 gu [M, 2F] contiguous; not under
    ``BPE_FP8_GEMM=lib``."""
    M, K = g.shape
    F = w8t.shape[0]
    return (_SWIGLU_BWD_GEMM and _MODE != "lib" and M % 256 == 0 and F % 256 == 0 and K % 128 == 0
            and K * 256 < 2**32 and F * K < 2**32 and w8t.is_contiguous() and w8t.dtype == FP8
            and gu.dtype == torch.bfloat16 and gu.is_contiguous() and tuple(gu.shape) == (M, 2 * F))


def grads_swiglu(g_state: Fp8State, g: Tensor, g_slot: int, w8t: Tensor, w_state: Fp8State, w_slot: int,
                 xt8: Tensor, x_state: Fp8State, x_slot: int, dw_out: Tensor | None, gu: Tensor, d_slot: int):
    """:func:`grads` for the W2 projection with the SwiGLU backward fused into its input gradient: ONE e5m2 cast of
    g (both layouts) feeds the weight gradient (accumulated into ``dw_out``, or returned) and the hand kernel that
    forms da = g @ W2 without storing it, applies the SwiGLU backward over ``gu`` and writes [dg | du] only as e5m2
    in both layouts (slot ``d_slot`` of ``g_state``; csrc/gemm_pp.hip EPI_SWIGLU_BWD8) -- the values of
    :func:`grads` + :func:`swiglu_bwd_cast_t` on the hand kernel.  Returns ``((dgu8, dgu8t), dW or None)``."""
    g = g.contiguous()
    if _t_ok(g):
        g8, g8t = g_state.cast_t(g, g_slot)
    else:
        g8 = g_state.cast(g, g_slot)
        g8t = g8.t().contiguous()
    gi = g_state.inv_scale[g_slot]
    M, F = g8.shape[0], w8t.shape[0]
    dgu8 = torch.empty(M, 2 * F, dtype=g_state.dtype, device=g.device)
    dgu8t = torch.empty(2 * F, M, dtype=g_state.dtype, device=g.device)
    ops().gemm_fp8_swiglu_bwd(g8, w8t, g_state.inv_scale[g_slot : g_slot + 1], w_state.inv_scale[w_slot : w_slot + 1],
                              gu, g_state.scale[d_slot : d_slot + 1], dgu8, dgu8t, g_state.amax[d_slot : d_slot + 1])
    if dw_out is not None:
        wgrad_acc(g8t, xt8, gi, x_state.inv_scale[x_slot], dw_out)
        return (dgu8, dgu8t), None
    return (dgu8, dgu8t), mm_fp8(g8t, xt8, gi, x_state.inv_scale[x_slot])


def swiglu_bwd_cast_t(state: Fp8State, da: Tensor, gu: Tensor, slot: int) -> tuple[Tensor, Tensor]:
    """The SwiGLU gate gradient [dg | du] from da [M, F] and gu [M, 2F], written only in fp8 (e5m2) in both layouts
    (dgu8 [M, 2F], dgu8t [2F, M]; slot ``slot``): one pass instead of ``swiglu_bwd`` plus ``cast_t``."""
    M, F2 = gu.shape
    g8 = torch.empty(M, F2, dtype=state.dtype, device=gu.device)
    g8t = torch.empty(F2, M, dtype=state.dtype, device=gu.device)
    ops().swiglu_cast_fp8_t(gu, da.contiguous(), state.scale[slot : slot + 1], g8, g8t, state.amax[slot : slot + 1])
    return g8, g8t


def norm_cast_ok(x: Tensor) -> bool:
    """A block input the fused residual add + RMSNorm + two-layout e4m3 cast takes: bf16 [M, N] contiguous, M and N
    multiples of 128, N <= 2048."""
    return (x.dtype == torch.bfloat16 and x.dim() == 2 and x.is_contiguous() and x.shape[0] % 128 == 0
            and x.shape[1] % 128 == 0 and x.shape[1] <= 2048)


def add_rmsnorm_cast_t(state: Fp8State, x: Tensor, d: Tensor | None, w: Tensor, eps: float, slot: int):
    """``s = x + d`` (``d`` None: ``s = x``) and ``RMSNorm(s) * w`` written only in fp8 (this state's e4m3) in both
    layouts, slot ``slot``: returns ``(s, (y8 [M, N], y8t [N, M]), rstd)``.  One pass for the norm (no bf16 y) plus
    an fp8 transpose, instead of ``add_rmsnorm_fwd`` and ``cast_t`` (csrc/fp8.hip add_rmsnorm_fp8_kernel)."""
    M, N = x.shape
    y8 = torch.empty(M, N, dtype=state.dtype, device=x.device)
    y8t = torch.empty(N, M, dtype=state.dtype, device=x.device)
    s, rstd = ops().add_rmsnorm_cast_fp8_t(x, None if d is None else d.contiguous(), w, eps,
                                           state.scale[slot : slot + 1], y8, y8t, state.amax[slot : slot + 1])
    return (x if d is None else s), (y8, y8t), rstd


def quantize_reference(x: Tensor, scale: float, fmt: str = "e4m3") -> Tensor:
    """Oracle: saturating cast to e4m3fn / e5m2 and back (for tests)."""
    dt, _ = _FMT[fmt]
    m = 448.0 if fmt == "e4m3" else 57344.0
    return (x.float() * scale).clamp(-m, m).to(dt).float() / scale
