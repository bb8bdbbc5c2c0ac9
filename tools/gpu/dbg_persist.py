# repeated one-tile vs persistent runs of a 297-tile GEMM (+ SwiGLU fwd / bwd): any run differing from the first
# one-tile result is reported with its tile coordinates
import sys
import torch
sys.path.insert(0, '.')
from bpe_transformer.ops._ext import ops
h = ops()
torch.manual_seed(5)
M, d, F = 8448, 768, 1024
x = torch.randn(M, d, device='cuda', dtype=torch.bfloat16)
w = (0.05 * torch.randn(2304, d, device='cuda')).to(torch.bfloat16)
w13 = (0.05 * torch.randn(2 * F, d, device='cuda')).to(torch.bfloat16)
w2 = (0.05 * torch.randn(d, F, device='cuda')).to(torch.bfloat16)
dy = torch.randn(M, d, device='cuda', dtype=torch.bfloat16)
base = None
nbad = 0
for it in range(8):
    for mode in (0, 1, 3):
        h.gpp_persist_config(mode)
        c = torch.empty(M, 2304, device='cuda', dtype=torch.bfloat16)
        h.gemm_pp(x, True, w, True, c, 0.0, 1)
        gu, a = h.gemm_swiglu_fwd(x, w13)
        dgu = h.gemm_swiglu_bwd(dy, w2, gu)
        out = (c, gu, a, dgu)
        if base is None:
            base = out
            continue
        for name, t0, t1 in zip(("plain", "gu", "act", "dgu"), base, out):
            if not torch.equal(t0, t1):
                nbad += 1
                dd = (t0 != t1)
                rows = dd.any(1).nonzero().flatten()
                print(f"iter {it} mode {mode} {name}: {dd.sum().item()} differ, rows {rows.min().item()}-{rows.max().item()}")
h.gpp_persist_config(0)
print("mismatching runs:", nbad)
