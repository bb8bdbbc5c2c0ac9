"""FP8 (OCP e4m3fn) forward projections with delayed per-tensor scaling.

Recipe (BASELINE.json "Llama-style 1.1B fp8 MFMA path"):
  * the four projection GEMMs of every block run as fp8 x fp8 -> bf16 on the
    MFMA fp8 units (hipBLASLt via ``torch._scaled_mm``, measured ~2x the bf16
    rate on MI355X at the 1.1B shapes, ``benchmarks/fp8_probe.py``);
  * activations and weights are quantised by ``csrc/fp8.hip`` with a scale
    derived from an amax history (delayed scaling, powers of two); the cast
    pass also records this step's amax, and one launch per step refreshes all
    scales -- the host never reads a scale;
  * backward GEMMs stay bf16 on the saved bf16 activations (fp8 forward,
    bf16 gradients), master weights and optimizer state stay fp32.
"""

from __future__ import annotations

import torch
from torch import Tensor

from ._ext import ops

FP8 = torch.float8_e4m3fn


class Fp8State:
    """Scaling state for ``n_slots`` quantised tensors (device-resident)."""

    def __init__(self, n_slots: int, device, history: int = 16, margin: float = 1.0):
        self.n = n_slots
        self.amax = torch.zeros(n_slots, dtype=torch.int32, device=device)
        self.hist = torch.zeros(n_slots, history, dtype=torch.float32, device=device)
        self.scale = torch.ones(n_slots, dtype=torch.float32, device=device)
        self.inv_scale = torch.ones(n_slots, dtype=torch.float32, device=device)
        self.margin = margin
        self.pos = 0

    def cast(self, x: Tensor, slot: int) -> Tensor:
        out = torch.empty(x.shape, dtype=FP8, device=x.device)
        ops().cast_fp8(x.contiguous(), self.scale[slot : slot + 1], out, self.amax[slot : slot + 1])
        return out

    def update(self) -> None:
        """Fold this step's amaxes into the history and recompute every scale (one launch)."""
        ops().update_scales(self.amax, self.hist, self.scale, self.inv_scale, self.pos, self.margin)
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

    def matmul(self, x: Tensor, w: Tensor, x_slot: int, w_slot: int) -> Tensor:
        """``x @ w.T`` in fp8 with bf16 output; x: [M, K] bf16, w: [N, K] bf16."""
        x8 = self.cast(x, x_slot)
        w8 = self.cast(w, w_slot)
        return torch._scaled_mm(x8, w8.t(), scale_a=self.inv_scale[x_slot], scale_b=self.inv_scale[w_slot],
                                out_dtype=torch.bfloat16)


def quantize_reference(x: Tensor, scale: float) -> Tensor:
    """Oracle: saturating cast to e4m3fn and back (for tests)."""
    return (x.float() * scale).clamp(-448.0, 448.0).to(FP8).float() / scale
