"""Noam learning-rate schedule (reference: distributed_training_transformer/
__main__.py:56-70): lr(step) = d_model^-0.5 * min(step * warmup^-1.5, step^-0.5).

Keras evaluates the schedule at `optimizer.iterations`, which starts at 0, so
the very first update uses lr = min(0, rsqrt(0) = inf) = 0; reproduced here.
The GPU optimizer evaluates the same formula on device (csrc/kernels/adam.hip).
"""
from __future__ import annotations

import math


def noam_lr(step: float, d_model: int, warmup: float = 4000.0) -> float:
    rise = step * warmup ** -1.5
    fall = math.inf if step <= 0 else step ** -0.5
    return d_model ** -0.5 * min(rise, fall)


class NoamSchedule:
    def __init__(self, d_model: int, warmup: float = 4000.0):
        self.d_model = d_model
        self.warmup = warmup

    def __call__(self, step: float) -> float:
        return noam_lr(step, self.d_model, self.warmup)
