"""The 4-wave persistent GEMM (``csrc/gemm_w4.hip``) against fp32 products of the same operands.

Small-integer operands make every output exact, so any layout, swizzle, stage-parity or seam slip shows as a
mismatch; the grid-cap fixture forces several tiles per workgroup (the K-tile sequence running across tile seams,
with odd and even K-tile counts), which is where the persistent pipeline's prefetch and store overlap live.
"""

from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.fixture(params=[(0, 1), (1, 1), (3, 1), (0, 0), (3, 0), (0, 2), (1, 2), (3, 2)],
                ids=["ring-percu", "ring-one_wg", "ring-three_wg", "2stage-percu", "2stage-three_wg", "regring-percu",
                     "regring-one_wg", "regring-three_wg"])
def w4_cap(request, gpu_device):
    """(workgroup cap, form): cap 0 = one per CU (the production form), 1 = a single workgroup walks every tile, 3 =
    tiles split unevenly over three; form 1 = the 4-stage ring of 32-deep steps, 0 = the 2-stage 64-deep form, 2 = the
    ring with register-staged loads."""
    h = torch.ops.bpe_hip
    cap, ring = request.param
    prev = h.gw4_grid_config(cap)
    prev_ring = h.gw4_ring_config(ring)
    yield request.param
    h.gw4_grid_config(prev)
    h.gw4_ring_config(prev_ring)


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("R", [448, 128, 192, 768])  # 7 / 2 / 3 / 12 K-tiles
def test_gemm_w4_exact(gpu_device, w4_cap, a_k, b_k, R):
    torch.manual_seed(R)
    M, N = 512, 768
    A = torch.randint(-1, 2, (M, R), device=gpu_device).to(torch.bfloat16)
    B = torch.randint(-1, 2, (N, R), device=gpu_device).to(torch.bfloat16)
    Am = A if a_k else A.t().contiguous()
    Bm = B if b_k else B.t().contiguous()
    C = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
    torch.ops.bpe_hip.gemm_w4(Am, a_k, Bm, b_k, C, 0.0)
    ref = A.float() @ B.float().t()
    assert torch.equal(C.float().cpu(), ref.cpu())


@pytest.mark.parametrize("a_k,b_k", [(True, True), (False, False)])
def test_gemm_w4_beta(gpu_device, w4_cap, a_k, b_k):
    torch.manual_seed(7)
    M, N, R = 768, 512, 320
    A = torch.randint(-1, 2, (M, R), device=gpu_device).to(torch.bfloat16)
    B = torch.randint(-1, 2, (N, R), device=gpu_device).to(torch.bfloat16)
    Am = A if a_k else A.t().contiguous()
    Bm = B if b_k else B.t().contiguous()
    C = torch.randint(-3, 4, (M, N), device=gpu_device).to(torch.bfloat16)
    ref = C.float() * 2.0 + A.float() @ B.float().t()
    torch.ops.bpe_hip.gemm_w4(Am, a_k, Bm, b_k, C, 2.0)
    assert torch.equal(C.float().cpu(), ref.cpu())


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, False)])
def test_gemm_w4_random(gpu_device, a_k, b_k):
    torch.manual_seed(0)
    M, N, R = 1024, 512, 1536
    A = torch.randn(M, R, device=gpu_device, dtype=torch.bfloat16)
    B = torch.randn(N, R, device=gpu_device, dtype=torch.bfloat16)
    Am = A if a_k else A.t().contiguous()
    Bm = B if b_k else B.t().contiguous()
    C = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
    torch.ops.bpe_hip.gemm_w4(Am, a_k, Bm, b_k, C, 0.0)
    ref = A.float() @ B.float().t()
    assert rel(C.cpu(), ref.cpu()) < 1e-2


def test_gemm_w4_bitwise_many_tiles(gpu_device):
    """297 tiles over 256 workgroups and over one, in both forms: the same per-tile MFMA order (k ascending), so
    bitwise-equal outputs, and repeated runs equal (no race between the seam prefetch, the epilogue stores and the
    next tile's reads)."""
    h = torch.ops.bpe_hip
    torch.manual_seed(5)
    M, d, N = 8448, 768, 2304
    x = torch.randn(M, d, device=gpu_device, dtype=torch.bfloat16)
    w = (0.05 * torch.randn(N, d, device=gpu_device)).to(torch.bfloat16)
    outs = []
    prev = h.gw4_grid_config(0)
    prev_ring = h.gw4_ring_config(1)
    try:
        for cap, ring in ((0, 1), (1, 1), (0, 1), (0, 1), (0, 0), (1, 0), (0, 2), (1, 2), (0, 2)):
            h.gw4_grid_config(cap)
            h.gw4_ring_config(ring)
            c = torch.empty(M, N, device=gpu_device, dtype=torch.bfloat16)
            h.gemm_w4(x, True, w, True, c, 0.0)
            outs.append(c)
    finally:
        h.gw4_grid_config(prev)
        h.gw4_ring_config(prev_ring)
    for c in outs[1:]:
        assert torch.equal(c, outs[0])
    assert rel(outs[0].cpu(), (x.float() @ w.float().t()).cpu()) < 1e-2
