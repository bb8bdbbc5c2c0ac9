"""Driver for the tile-order counter runs (profiles/pmc/gemm_tile_order_pmc_r6.md): the GPT-2 B 128 SwiGLU-forward,
plain W13 and QKV + RoPE GEMMs at tile order gm 0 and gm 4 (gpp_order_config), three rounds, dispatch order
fixed (swiglu, w13, qkv) x (gm 0, gm 4) per round.  Run it under rocprofv3 --kernel-trace / --pmc."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from bpe_transformer.ops._ext import ops
h = ops()
M, d, F = 131072, 768, 2048
torch.manual_seed(0)
x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
w13 = (0.05 * torch.randn(2 * F, d, device="cuda")).to(torch.bfloat16)
wq = (0.05 * torch.randn(3 * d, d, device="cuda")).to(torch.bfloat16)
S, D = 1024, 64
cos = torch.randn(S, D // 2, device="cuda"); sin = torch.randn(S, D // 2, device="cuda")
c2 = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
torch.cuda.synchronize()
# dispatch order per round: gm 0 then gm 4 (swiglu fwd, w13 plain, qkv rope), three rounds
for _ in range(3):
    for gm in (0, 4):
        h.gpp_order_config(gm)
        h.gemm_swiglu_fwd(x, w13)
        h.gemm_pp(x, True, w13, True, c2, 0.0, 1)
        h.gemm_qkv_rope(x, wq, cos, sin, S, D, 2 * d)
torch.cuda.synchronize()
