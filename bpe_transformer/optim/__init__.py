"""Optimizers, gradient clipping and learning-rate schedules."""

from ..ops.optim import clip_grad_norm_
from .adamw import AdamW
from .flat import FlatAdamW, FlatParameters
from .schedule import CosineSchedule, get_lr_cosine_schedule

gradient_clipping = clip_grad_norm_

__all__ = ["AdamW", "CosineSchedule", "FlatAdamW", "FlatParameters", "clip_grad_norm_", "get_lr_cosine_schedule",
           "gradient_clipping"]
