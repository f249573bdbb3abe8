"""Ready-made hyperparameter schedules (reference ``kfac/hyperparams.py``)."""
from __future__ import annotations

from typing import Callable


def exp_decay_factor_averaging(
    min_value: float = 0.95,
) -> Callable[[int], float]:
    """Running-average weight schedule ``k -> min(1 - 1/k, min_value)``.

    Early in training the running average behaves like a plain mean of the
    factors seen so far (weight ``1 - 1/k``); after ``1/(1-min_value)`` steps
    it becomes an exponential moving average with weight ``min_value``.
    Step 0 is treated as step 1 and negative steps raise ``ValueError``
    (reference ``kfac/hyperparams.py:7-46``).

    Returns:
        callable usable as ``factor_decay`` of a preconditioner.
    """
    if min_value <= 0:
        raise ValueError('min_value must be greater than 0')

    def schedule(step: int) -> float:
        if step < 0:
            raise ValueError(f'step value cannot be negative. Got step={step}.')
        k = max(step, 1)
        return min(1.0 - 1.0 / k, min_value)

    return schedule
