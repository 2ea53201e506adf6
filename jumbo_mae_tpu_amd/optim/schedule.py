"""Learning-rate schedules with optax semantics.

Parity: ``optax.warmup_cosine_decay_schedule(init_value=1e-6, peak, warmup_steps,
decay_steps=training_steps, end_value)`` as used by the reference
(/root/reference/src/pretraining.py:253-259, finetuning.py:257-263).  optax joins a linear
warmup with a cosine decay over ``decay_steps - warmup_steps`` steps (quirk Q17: the cosine
runs over training_steps - warmup_steps), alpha = end_value / peak_value.
Step ``count`` starts at 0 (``inject_hyperparams`` evaluates the schedule at the optimizer's
count before incrementing it).
"""

from __future__ import annotations

import math
from dataclasses import dataclass


@dataclass(frozen=True)
class WarmupCosine:
    init_value: float
    peak_value: float
    warmup_steps: int
    decay_steps: int
    end_value: float = 0.0

    def __call__(self, count: int) -> float:
        count = float(count)
        if self.warmup_steps > 0 and count < self.warmup_steps:
            frac = 1.0 - max(0.0, min(count, self.warmup_steps)) / self.warmup_steps
            return (self.init_value - self.peak_value) * frac + self.peak_value
        steps = self.decay_steps - self.warmup_steps
        c = count - self.warmup_steps
        alpha = 0.0 if self.peak_value == 0 else self.end_value / self.peak_value
        if steps <= 0:
            return self.peak_value  # optax returns init_value of the cosine part
        c = min(max(c, 0.0), steps)
        cosine = 0.5 * (1.0 + math.cos(math.pi * c / steps))
        return self.peak_value * ((1.0 - alpha) * cosine + alpha)

    def as_tuple(self) -> tuple[float, float, float, float, float]:
        return (self.init_value, self.peak_value, float(self.warmup_steps), float(self.decay_steps),
                self.end_value)


def warmup_cosine_decay_schedule(init_value: float, peak_value: float, warmup_steps: int,
                                 decay_steps: int, end_value: float = 0.0) -> WarmupCosine:
    return WarmupCosine(init_value, peak_value, int(warmup_steps), int(decay_steps), end_value)
