"""Learning-rate schedules.

Cosine with linear warmup: reference contract K16 (``tests/adapters.py:477-502``,
expected values ``tests/test_optimizer.py:58-84``):
  it < Tw:          it / Tw * max
  Tw <= it <= Tc:   min + 0.5 * (1 + cos(pi * (it - Tw) / (Tc - Tw))) * (max - min)
  it > Tc:          min
"""

from __future__ import annotations

import math


def get_lr_cosine_schedule(it: int, max_learning_rate: float, min_learning_rate: float, warmup_iters: int,
                           cosine_cycle_iters: int) -> float:
    if it < warmup_iters:
        return it / warmup_iters * max_learning_rate
    if it <= cosine_cycle_iters:
        span = max(cosine_cycle_iters - warmup_iters, 1)
        frac = (it - warmup_iters) / span
        return min_learning_rate + 0.5 * (1.0 + math.cos(math.pi * frac)) * (max_learning_rate - min_learning_rate)
    return min_learning_rate


class CosineSchedule:
    def __init__(self, max_lr: float, min_lr: float, warmup_iters: int, cosine_cycle_iters: int):
        self.max_lr, self.min_lr = max_lr, min_lr
        self.warmup_iters, self.cosine_cycle_iters = warmup_iters, cosine_cycle_iters

    def __call__(self, it: int) -> float:
        return get_lr_cosine_schedule(it, self.max_lr, self.min_lr, self.warmup_iters, self.cosine_cycle_iters)
