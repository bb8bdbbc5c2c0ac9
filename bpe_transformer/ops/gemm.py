"""Weight-gradient GEMMs (``g += dy^T @ x``) on the hand-written gfx950 kernels.

``accumulate_weight_grad(g, dy, x)`` computes ``g += dy^T @ x`` where
``dy: [T, N]`` and ``x: [T, K]`` are token-major activations (T = batch*seq)
and ``g: [N, K]`` is a view of the flat bf16 gradient buffer.  The reduction
runs over all T tokens, which for a training step is large (16k-128k) while
N x K is small: the kernels split T across workgroups (enough to fill all 256
CUs) and reduce the fp32 partials deterministically into ``g``.

Routes per shape (``_run``; the measured choice per training shape is in ``tuning/dw_routes.json``):

* ``pp``  -- the 8-wave ping-pong kernel (``csrc/gemm_pp.hip``), both operands token-major;
* ``ppt`` -- the same kernel on a transposed copy of X (B K-major);
* ``hip256`` / ``hip128`` -- the 256 x 256 and 128 x 128 split-K kernels of ``csrc/gemm.hip``;
* ``blas`` -- hipBLASLt (``addmm_``), for shapes none of the HIP kernels covers.

``accumulate_weight_grads(items)`` runs the dW GEMMs of one layer that are ready at the same time as ONE grouped
split-K launch (``gemm_pp_dw_group``: the ping-pong kernel over the concatenated tile lists, one ordered reduce),
so that tiles x splits fills whole waves of the 256 CUs for the set instead of for each shape alone.
"""

from __future__ import annotations

import json
import os

import torch
from torch import Tensor

from ._ext import ops

# split-K target workgroups of the 128-tile kernel (256 / 768 / 1024 measured within noise of 512:
# profiles/bench/ab_gemm_target_wgs_b128.log)
_TARGET_WGS = 512


def choose_splits(n: int, k: int, t: int, target: int = _TARGET_WGS, min_iters: int = 8) -> int:
    tiles = (n // 128) * (k // 128)
    best = 1
    s = 1
    while s <= 64:
        if t % (64 * s) == 0 and t // (64 * s) >= min_iters:
            best = s
            if tiles * s >= target:
                break
        s *= 2
    return best


_MAX_TILES = 160  # the 128-tile kernel's output-tile cap (256 measured the same: ab_gemm_target_wgs_b128.log)
_CUS = 256


def choose_splits_256(n: int, k: int, t: int) -> int:
    """Split count for the 256-tile kernel from a wave-quantised cost model.

    time(s) ~ ceil(tiles*s / CUs) * (t/s/32) * t_kstep  +  (s > 1) * slab traffic (s*n*k fp32 written + read).
    One workgroup per CU, so the grid runs in ceil(tiles*s/256) waves of equal length.
    """
    tiles = (n // 256) * (k // 256)
    nk = t // 32
    t_kstep = 0.8e-6  # one 256x256x32 MFMA step at ~50% of the dense bf16 rate
    best, best_cost = 1, None
    for s in range(1, 65):
        if nk // s < 8:
            continue
        # split ranges may be uneven (the kernel gives split i steps [i*nk/s, (i+1)*nk/s)); a wave lasts as long
        # as its longest split
        waves = -(-tiles * s // _CUS)
        cost = waves * (-(-nk // s)) * t_kstep + (2 * s * n * k * 4 / 4.0e12 if s > 1 else 0.0)
        if best_cost is None or cost < best_cost * 0.97:
            best, best_cost = s, cost
    return best


def use_tile256(n: int, k: int, t: int) -> bool:
    return n % 256 == 0 and k % 256 == 0 and t % 256 == 0


def supported(n: int, k: int, t: int) -> bool:
    """Shapes routed to the split-K kernel: tile-aligned and with few output tiles.

    Measured on MI355X (benchmarks/gemm_bench.py, 16k and 64k tokens): the split-K kernel beats hipBLASLt
    1.25-1.67x on the 768x768 / 2304x768 / 768x2048 gradients (36-108 tiles of 128x128) and loses ~10% on
    the 4096x768 one (192 tiles), where the library's own tiles already fill the chip.
    """
    return n % 128 == 0 and k % 128 == 0 and t % 64 == 0 and (n // 128) * (k // 128) <= _MAX_TILES


_AUTOTUNE = os.environ.get("BPE_GEMM_AUTOTUNE", "1") == "1"
_route: dict[tuple[int, int, int], str] = {}
_ROUTES_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning", "dw_routes.json")


def _load_static_routes(path: str | None = None) -> dict[tuple[int, int, int], str]:
    """Measured per-shape dW routes (``tuning/dw_routes.json``: ``"N,K,T": route``), so a known training shape gets
    the same kernel -- and the same numerics -- on every run and every rank.  ``BPE_GEMM_ROUTES`` = another table,
    or ``off`` to time every shape at first use."""
    path = path or os.environ.get("BPE_GEMM_ROUTES", _ROUTES_FILE)
    if path == "off" or not os.path.exists(path):
        return {}
    with open(path) as f:
        raw = json.load(f)
    return {tuple(int(v) for v in k.split(",")): r for k, r in raw.get("routes", raw).items()}


_static_route = _load_static_routes()


def choose_splits_pp(n: int, k: int, t: int, cus: int = _CUS) -> int:
    """Split count for the ping-pong kernel (256 x 256 x 64 tiles): fill whole waves of CUs, keep >= 4 K-tiles
    per split, and charge the fp32 slab round trip."""
    tiles = (n // 256) * (k // 256)
    nk = t // 64
    best, best_cost = 1, None
    for s in range(1, 65):
        if nk // s < 4:
            break
        waves = -(-tiles * s // cus)
        cost = waves * (-(-nk // s)) * 1.6e-6 + (2 * s * n * k * 4 / 4.0e12 if s > 1 else 0.0)
        if best_cost is None or cost < best_cost * 0.97:
            best, best_cost = s, cost
    return best


def use_pp(n: int, k: int, t: int) -> bool:
    return n % 256 == 0 and k % 256 == 0 and t % 64 == 0


def _candidates(n: int, k: int, t: int) -> list[str]:
    c = []
    if use_pp(n, k, t):
        c.append("pp")
        if t * 256 < 2**31:  # ppt's X^T [K][T] has leading dimension T (the kernel's 32-bit tile offsets)
            c.append("ppt")
    if use_tile256(n, k, t):
        c.append("hip256")
    elif supported(n, k, t):
        c.append("hip128")
    return c + ["blas"]


def _blas_acc(g: Tensor, dy: Tensor, x: Tensor) -> None:
    if g.dtype == dy.dtype:
        g.addmm_(dy.t(), x)
    else:  # fp32 gradient buffer, bf16 activations: fp32 product (no bf16 rounding of dW)
        g.addmm_(dy.t().to(g.dtype), x.to(g.dtype))


def _run(route: str, g: Tensor, dy: Tensor, x: Tensor, x_scale: Tensor | None = None) -> None:
    n, k = g.shape
    t = dy.shape[0]
    if x_scale is not None:
        if route == "ppt":  # the scale rides on the X^T copy the route makes anyway
            xt = ops().transpose_bf16(x, x_scale.detach().float().reshape(1).contiguous())
            ops().gemm_pp(dy, False, xt, True, g, 1.0, choose_splits_pp(n, k, t))
            return
        x = x * x_scale.to(x.dtype)
    if route == "pp":
        ops().gemm_pp(dy, False, x, False, g, 1.0, choose_splits_pp(n, k, t))
    elif route == "ppt":
        # X^T materialised (ops.transpose_bf16): B K-major, the ping-pong kernel's MN x K layout -- ahead of the
        # token-major x token-major one on the LM head (benchmarks/dw_ppt.py, profiles/bench/dw_ppt_r5.log)
        ops().gemm_pp(dy, False, ops().transpose_bf16(x), True, g, 1.0, choose_splits_pp(n, k, t))
    elif route == "hip256":
        ops().gemm(dy, False, x, False, g, 1.0, choose_splits_256(n, k, t), 256)
    elif route == "hip128":
        ops().gemm(dy, False, x, False, g, 1.0, choose_splits(n, k, t), 128)
    else:
        _blas_acc(g, dy, x)


_warned: set = set()


def _tune(key: tuple[int, int, int], cands: list[str], g: Tensor, dy: Tensor, x: Tensor) -> str:
    """Time each route once per shape on a scratch output (CUDA events, 3 reps) and keep the fastest.

    Single process only.  Under ``torch.distributed`` with more than one rank nothing is timed here: a timing
    inside the backward would need a host sync plus a collective in the middle of the step, and any rank whose
    environment or table differed would deadlock.  An off-table shape there takes the first HIP candidate (the same
    choice on every rank: it depends on the shape only) and a warning names the shape to add to
    ``tuning/dw_routes.json``.
    """
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if key not in _warned:
            _warned.add(key)
            import warnings

            warnings.warn(f"dW GEMM shape N,K,T={key} is not in ops/tuning/dw_routes.json; using route "
                          f"'{cands[0]}' without timing (multi-rank job)", stacklevel=3)
        return cands[0]
    if not _AUTOTUNE or len(cands) == 1 or torch.cuda.is_current_stream_capturing():
        return cands[0]
    scratch = torch.empty_like(g)
    times = []
    for c in cands:
        _run(c, scratch, dy, x)  # warm (kernel attributes, library heuristics)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3):
            _run(c, scratch, dy, x)
        e.record()
        e.synchronize()
        times.append(s.elapsed_time(e))
    return cands[min(range(len(cands)), key=lambda i: times[i])]


def weight_grad_route(n: int, k: int, t: int) -> str | None:
    """The route chosen for a dW shape (None until first use)."""
    return _route.get((n, k, t))


def routes_summary() -> dict[str, str]:
    """``{"N,K,T": route}`` for every dW shape used so far in this process (for metrics / bench output)."""
    return {",".join(str(v) for v in k): r for k, r in sorted(_route.items())}


def accumulate_weight_grad(g: Tensor, dy: Tensor, x: Tensor, x_scale: Tensor | None = None) -> None:
    """``g += dy.T @ (x_scale * x)`` (bf16 operands, fp32 accumulation; ``g`` bf16 or fp32 -- an fp32 gradient
    buffer gets the fp32 sum, through the kernels' fp32 partial slab and ordered reduce).  ``x_scale``: optional
    device scalar (the LM head's upstream loss gradient), folded into the X^T copy of the ``ppt`` route, else
    applied to x first.

    Routes per shape (module docstring): the shape's entry in ``tuning/dw_routes.json``, else the first call for a
    shape times the candidates (``BPE_GEMM_AUTOTUNE=0``: take the first HIP candidate).  Measured
    (benchmarks/gemm_dw.py, dw_ppt.py): the HIP kernels win every GPT-2-small dW shape 1.4-2.3x over hipBLASLt;
    hipBLASLt keeps Llama's 2048 x 5632 one at 16 384 tokens.
    """
    n, k = g.shape
    t = dy.shape[0]
    ok = (g.is_cuda and g.dtype in (torch.bfloat16, torch.float32) and dy.dtype == torch.bfloat16
          and x.dtype == torch.bfloat16 and g.stride(1) == 1 and dy.stride(1) == 1 and x.stride(1) == 1)
    if not ok:
        _blas_acc(g, dy, x if x_scale is None else x * x_scale.to(x.dtype))
        return
    key = (n, k, t) if g.dtype == torch.bfloat16 else (n, k, t, 32)
    route = _route.get(key)
    if route is None:
        cands = _candidates(n, k, t)
        if g.dtype == torch.float32 and len(cands) > 1:
            cands = cands[:-1]  # the HIP kernels write an fp32 C exactly; the library route would cast
        key3 = (n, k, t)
        fixed = _static_route.get(key3)
        route = _route[key] = fixed if fixed in cands else _tune(key3, cands, g, dy, x)
    _run(route, g, dy, x, x_scale)


def matmul_nt(a: Tensor, b: Tensor, out: Tensor | None = None, beta: float = 0.0) -> Tensor:
    """``out = beta*out + a @ b.T`` with a: [M, R], b: [N, R] (both K-major) on the HIP kernel."""
    m, r = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, device=a.device, dtype=a.dtype)
        beta = 0.0
    ops().gemm(a, True, b, True, out, beta, choose_splits(m, n, r), 128)
    return out


# ---------------------------------------------------------------------------------------------------------------
# Grouped weight gradients (one split-K launch for the dW GEMMs of a layer that become ready together)

_GROUP = os.environ.get("BPE_DW_GROUP", "0") == "1"  # opt-in: measured neutral at GPT-2, -2.2 % at Llama (profiles/bench/ab_dw_group_r6.log)
_group_used: dict[tuple, int] = {}


def choose_splits_group(tiles: int, t: int, mn: int, cus: int = _CUS) -> int:
    """Split count for a grouped launch of ``tiles`` 256 x 256 tiles over ``t`` tokens (``mn`` = sum of the output
    elements), in units of one K-tile of the loop: every wave of ``cus`` workgroups lasts as long as a split's
    K-tiles plus a fixed ~6.5 K-tiles (prologue round trip + the 256 KiB fp32 slab store; per-workgroup stamps,
    profiles/bench/dw_stamps_r6.log), and the slab round trip through HBM costs ~8 bytes per element per split."""
    nk = t // 64
    best, best_cost = 1, None
    for s in range(1, 65):
        if nk // s < 8:
            break
        waves = -(-tiles * s // cus)
        cost = waves * (-(-nk // s) + 6.5) + (s * mn * 8.4e-7 if s > 1 else 0.0)
        if best_cost is None or cost < best_cost * 0.99:
            best, best_cost = s, cost
    return best


def _group_ok(items: list[tuple[Tensor, Tensor, Tensor]]) -> bool:
    if not (2 <= len(items) <= 4):
        return False
    g0, dy0, _ = items[0]
    t = dy0.shape[0]
    if not (g0.is_cuda and g0.dtype in (torch.bfloat16, torch.float32) and t % 64 == 0 and t * 256 < 2**31):
        return False
    for g, dy, x in items:
        n, k = g.shape
        if not (g.dtype == g0.dtype and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
                and g.device == g0.device and dy.shape == (t, n) and x.shape == (t, k) and n % 256 == 0
                and k % 256 == 0 and g.stride(1) == 1 and dy.stride(1) == 1 and x.stride(1) == 1
                and g.stride(0) % 8 == 0 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0
                and dy.stride(0) * 256 < 2**31 and x.stride(0) * 256 < 2**31
                and g.data_ptr() % 16 == 0 and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0):
            return False
    return True


def accumulate_weight_grads(items: list[tuple[Tensor, Tensor, Tensor]]) -> None:
    """``g += dy^T @ x`` for every ``(g, dy, x)`` of ``items`` (the same token count T for all).

    Two to four eligible shapes (256-multiples, bf16 operands, all-bf16 or all-fp32 gradients) run as one grouped
    split-K launch of the ping-pong kernel plus one ordered reduce (``gemm_pp_dw_group``); the split count is chosen
    for the set (:func:`choose_splits_group`), so the result is deterministic and depends on the shapes only (the
    same on every rank).  Otherwise -- or with ``BPE_DW_GROUP=0`` -- each item takes its per-shape route."""
    if _GROUP and _group_ok(items):
        t = items[0][1].shape[0]
        tiles = sum((g.shape[0] // 256) * (g.shape[1] // 256) for g, _, _ in items)
        mn = sum(g.numel() for g, _, _ in items)
        s = choose_splits_group(tiles, t, mn)
        key = tuple((g.shape[0], g.shape[1]) for g, _, _ in items) + (t,)
        _group_used[key] = s
        ops().gemm_pp_dw_group([g for g, _, _ in items], [dy for _, dy, _ in items], [x for _, _, x in items],
                               False, s, 1.0)
        return
    for g, dy, x in items:
        accumulate_weight_grad(g, dy, x)


def groups_summary() -> dict[str, int]:
    """``{"N,K+N,K+...,T": splits}`` for every grouped dW launch so far in this process (bench output)."""
    return {"+".join(f"{n},{k}" for n, k in key[:-1]) + f",{key[-1]}": s for key, s in sorted(_group_used.items())}
