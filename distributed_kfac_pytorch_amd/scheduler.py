"""Multiplicative hyperparameter scheduler (reference ``kfac/scheduler.py``).

``LambdaParamScheduler.step()`` multiplies each targeted hyperparameter of a
preconditioner by ``lambda(step)``.  Like the reference (``scheduler.py:
118-166``) the update COMPOUNDS across calls and the two step-count
hyperparameters are truncated to ``int`` after each multiplication.
"""
from __future__ import annotations

from typing import Callable
from typing import TYPE_CHECKING

if TYPE_CHECKING:  # pragma: no cover
    from distributed_kfac_pytorch_amd.base_preconditioner import (
        BaseKFACPreconditioner,
    )

# (constructor keyword, private attribute on the preconditioner, int-cast)
_TARGETS: tuple[tuple[str, str, bool], ...] = (
    ('factor_update_steps', '_factor_update_steps', True),
    ('inv_update_steps', '_inv_update_steps', True),
    ('damping', '_damping', False),
    ('factor_decay', '_factor_decay', False),
    ('kl_clip', '_kl_clip', False),
    ('lr', '_lr', False),
)


class LambdaParamScheduler:
    """Scale preconditioner hyperparameters by user lambdas of the step."""

    def __init__(
        self,
        preconditioner: BaseKFACPreconditioner,
        *,
        factor_update_steps_lambda: Callable[[int], float] | None = None,
        inv_update_steps_lambda: Callable[[int], float] | None = None,
        damping_lambda: Callable[[int], float] | None = None,
        factor_decay_lambda: Callable[[int], float] | None = None,
        kl_clip_lambda: Callable[[int], float] | None = None,
        lr_lambda: Callable[[int], float] | None = None,
    ) -> None:
        """Init LambdaParamScheduler.

        Raises:
            ValueError: if a lambda targets a hyperparameter that is already a
                callable on the preconditioner (it cannot be multiplied).
        """
        self._preconditioner = preconditioner
        given = {
            'factor_update_steps': factor_update_steps_lambda,
            'inv_update_steps': inv_update_steps_lambda,
            'damping': damping_lambda,
            'factor_decay': factor_decay_lambda,
            'kl_clip': kl_clip_lambda,
            'lr': lr_lambda,
        }
        self._lambdas: list[tuple[str, bool, Callable[[int], float]]] = []
        for name, attr, as_int in _TARGETS:
            fn = given[name]
            if fn is None:
                continue
            if callable(getattr(preconditioner, attr)):
                raise ValueError(
                    f'preconditioner.{name} is already a callable and cannot '
                    'be updated by the lambdaparamscheduler.',
                )
            self._lambdas.append((attr, as_int, fn))

    def step(self, step: int | None = None) -> None:
        """Apply every lambda once (call after ``preconditioner.step()``).

        Args:
            step (int, optional): value passed to the lambdas instead of the
                preconditioner's current step.
        """
        p = self._preconditioner
        k = p.steps if step is None else step
        for attr, as_int, fn in self._lambdas:
            current = getattr(p, attr)
            assert not callable(current)
            value = current * fn(k)
            setattr(p, attr, int(value) if as_int else value)
