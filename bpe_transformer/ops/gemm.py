"""Hand-written gfx950 split-K MFMA GEMMs (``csrc/gemm.hip``) for weight gradients.

``accumulate_weight_grad(g, dy, x)`` computes ``g += dy^T @ x`` where
``dy: [T, N]`` and ``x: [T, K]`` are token-major activations (T = batch*seq)
and ``g: [N, K]`` is a view of the flat bf16 gradient buffer.  The reduction
runs over all T tokens, which for a training step is large (16k-64k) while
N x K is small: the kernel splits T across workgroups (enough to fill all 256
CUs) and reduces the fp32 partials deterministically into ``g``.

Two kernels: the 256 x 256 tile (8 waves, LDS-DMA staging, one workgroup per
CU) for shapes that are multiples of 256, the 128 x 128 tile otherwise.
Shapes neither covers go to hipBLASLt (``addmm_``).
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
        c += ["pp", "ppt"]
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


def _run(route: str, g: Tensor, dy: Tensor, x: Tensor) -> None:
    n, k = g.shape
    t = dy.shape[0]
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


def accumulate_weight_grad(g: Tensor, dy: Tensor, x: Tensor) -> None:
    """``g += dy.T @ x`` (bf16 operands, fp32 accumulation; ``g`` bf16 or fp32 -- an fp32 gradient buffer gets the
    fp32 sum, through the kernels' fp32 partial slab and ordered reduce).

    Routes per shape between the 256-tile HIP kernel, the 128-tile HIP kernel and hipBLASLt; the first call
    for a shape times the candidates (``BPE_GEMM_AUTOTUNE=0``: take the HIP kernel whenever it applies).
    Measured (benchmarks/gemm_dw.py): the HIP kernel wins every GPT-2-small dW shape 1.4-2.3x; hipBLASLt
    keeps Llama's 2048 x 5632 one.
    """
    n, k = g.shape
    t = dy.shape[0]
    ok = (g.is_cuda and g.dtype in (torch.bfloat16, torch.float32) and dy.dtype == torch.bfloat16
          and x.dtype == torch.bfloat16 and g.stride(1) == 1 and dy.stride(1) == 1 and x.stride(1) == 1)
    if not ok:
        _blas_acc(g, dy, x)
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
    _run(route, g, dy, x)


def matmul_nt(a: Tensor, b: Tensor, out: Tensor | None = None, beta: float = 0.0) -> Tensor:
    """``out = beta*out + a @ b.T`` with a: [M, R], b: [N, R] (both K-major) on the HIP kernel."""
    m, r = a.shape
    n = b.shape[0]
    if out is None:
        out = torch.empty(m, n, device=a.device, dtype=a.dtype)
        beta = 0.0
    ops().gemm(a, True, b, True, out, beta, choose_splits(m, n, r), 128)
    return out
