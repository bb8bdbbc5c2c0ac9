"""AdamW (decoupled weight decay), the reference contract K15
(``tests/adapters.py:470-474``; test ``tests/test_optimizer.py:29-49``).

Update per parameter (identical to ``torch.optim.AdamW``):
    p <- p * (1 - lr*wd);  m <- b1 m + (1-b1) g;  v <- b2 v + (1-b2) g^2
    p <- p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)

GPU parameters are updated by the fused HIP kernel (``ops.fused_adamw_step``);
bf16 parameters keep an fp32 master copy in the optimizer state, and the
kernel writes the rounded bf16 weights back in the same pass.  For whole-model
training use :class:`bpe_transformer.optim.flat.FlatAdamW`, which does the
entire step in one launch over flat buffers.
"""

from __future__ import annotations

import torch

from ..ops.optim import fused_adamw_step


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.01):
        if lr < 0:
            raise ValueError(f"invalid learning rate {lr}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas {betas}")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                state = self.state[p]
                if not state:
                    state["step"] = 0
                    state["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32,
                                                           memory_format=torch.contiguous_format)
                    if p.dtype != torch.float32:
                        state["master"] = p.detach().float().contiguous().clone()
                state["step"] += 1
                master = state.get("master")
                g = p.grad
                if master is None:
                    if p.is_contiguous():
                        fused_adamw_step(p.data, state["exp_avg"], state["exp_avg_sq"], g.contiguous(), None, lr, b1,
                                         b2, eps, wd, state["step"])
                    else:
                        tmp = p.data.contiguous()
                        fused_adamw_step(tmp, state["exp_avg"], state["exp_avg_sq"], g.contiguous(), None, lr, b1,
                                         b2, eps, wd, state["step"])
                        p.data.copy_(tmp)
                else:
                    out = p.data if (p.dtype == torch.bfloat16 and p.is_contiguous() and p.is_cuda) else None
                    fused_adamw_step(master, state["exp_avg"], state["exp_avg_sq"], g.contiguous(), out, lr, b1, b2,
                                     eps, wd, state["step"])
                    if out is None:
                        p.data.copy_(master)
        return loss
