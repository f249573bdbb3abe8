"""Execution tracing (reference ``kfac/tracing.py:18-107``) plus GPU phases.

Two layers:

* ``trace(sync=False)`` / ``get_trace`` / ``log_trace`` / ``clear_trace`` —
  the reference's wall-clock decorator API, unchanged in behaviour.
* ``PhaseTimer`` — MI355X-native per-phase timing with HIP events recorded
  on the current stream (no host sync while recording).  The preconditioner
  records ``factor``, ``reduce``, ``inverse``, ``broadcast``,
  ``precondition`` and ``apply`` phases into it when
  ``KFAC_PHASE_TIMING=1`` (or ``enable_phase_timing()``), and ``bench.py``
  reports them.  Ranges are also pushed to roctx (via ``torch.cuda.nvtx``,
  which maps to roctx on ROCm) so they show up in ``rocprofv3
  --marker-trace``.
"""
from __future__ import annotations

import contextlib
import logging
import os
import sys
import time
from collections import defaultdict
from typing import Any
from typing import Callable
from typing import Iterator
from typing import TypeVar

import torch

from distributed_kfac_pytorch_amd.utils.env import getenv

RT = TypeVar('RT')

_func_traces: dict[str, list[float]] = {}
logger = logging.getLogger(__name__)


def clear_trace() -> None:
    """Clear recorded traces globally."""
    _func_traces.clear()


def get_trace(
    average: bool = True,
    max_history: int | None = None,
) -> dict[str, float]:
    """Return ``{function name: mean (or summed) seconds}``.

    Args:
        average (bool): mean of the recorded times if True, else their sum.
        max_history (int, optional): only use the last ``max_history`` calls.
    """
    out: dict[str, float] = {}
    for fname, times in _func_traces.items():
        if max_history is not None and len(times) > max_history:
            times = times[-max_history:]
        total = sum(times)
        out[fname] = total / len(times) if average else total
    return out


def log_trace(
    average: bool = True,
    max_history: int | None = None,
    loglevel: int = logging.INFO,
) -> None:
    """Log the times recorded by ``@trace`` (see ``get_trace``)."""
    for fname, value in get_trace(average, max_history).items():
        logger.log(loglevel, f'{fname}: {value}')


def trace(
    sync: bool = False,
) -> Callable[[Callable[..., RT]], Callable[..., RT]]:
    """Decorator recording the wall time of each call of a function.

    Args:
        sync (bool): barrier all ranks before and after the call, so the
            recorded time is the slowest rank's.
    """

    def decorator(func: Callable[..., RT]) -> Callable[..., RT]:
        def timed(*args: Any, **kwargs: Any) -> RT:
            if sync:
                torch.distributed.barrier()
            t0 = time.time()
            out = func(*args, **kwargs)
            if sync:
                torch.distributed.barrier()
            _func_traces.setdefault(func.__name__, []).append(
                time.time() - t0,
            )
            return out

        timed.__name__ = func.__name__
        timed.__doc__ = func.__doc__
        return timed

    return decorator


class PhaseTimer:
    """HIP-event timer for the K-FAC phases of a step.

    ``with timer.phase('precondition'):`` records a start/stop event pair on
    the current stream.  Nothing blocks until ``summary()`` is called, which
    synchronizes once and converts every recorded pair to milliseconds.
    On CPU the timer falls back to ``time.perf_counter``.
    """

    def __init__(self) -> None:
        self._pending: list[tuple[str, Any, Any]] = []
        self._ms: dict[str, list[float]] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str) -> Iterator[None]:
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            start = torch.cuda.Event(enable_timing=True)
            stop = torch.cuda.Event(enable_timing=True)
            torch.cuda.nvtx.range_push(f'kfac:{name}')
            start.record()
            try:
                yield
            finally:
                stop.record()
                torch.cuda.nvtx.range_pop()
                self._pending.append((name, start, stop))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._ms[name].append((time.perf_counter() - t0) * 1e3)

    def _drain(self) -> None:
        if self._pending:
            torch.cuda.synchronize()
            for name, start, stop in self._pending:
                self._ms[name].append(start.elapsed_time(stop))
            self._pending.clear()

    def summary(self, average: bool = False) -> dict[str, float]:
        """Return ``{phase: total ms}`` (or mean ms per call)."""
        self._drain()
        out = {}
        for name, vals in self._ms.items():
            out[name] = sum(vals) / len(vals) if average else sum(vals)
        return out

    def counts(self) -> dict[str, int]:
        self._drain()
        return {k: len(v) for k, v in self._ms.items()}

    def reset(self) -> None:
        self._pending.clear()
        self._ms.clear()


_PHASE_TIMER: PhaseTimer | None = (
    PhaseTimer() if os.environ.get('KFAC_PHASE_TIMING') == '1' else None
)


def enable_phase_timing(enable: bool = True) -> PhaseTimer | None:
    """Turn the global K-FAC phase timer on or off; returns it."""
    global _PHASE_TIMER
    _PHASE_TIMER = PhaseTimer() if enable else None
    return _PHASE_TIMER


def phase_timer() -> PhaseTimer | None:
    """The global phase timer, or None when phase timing is off."""
    return _PHASE_TIMER


@contextlib.contextmanager
def phase(name: str) -> Iterator[None]:
    """Record a K-FAC phase on the global timer (no-op when disabled, and
    while a HIP graph is being captured: event timing is not capturable)."""
    timer = _PHASE_TIMER
    if getenv('KFAC_DEBUG_SYNC') == '1' and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        # KFAC_DEBUG_SYNC=1: synchronise after every phase so an asynchronous
        # device fault is reported by the phase that caused it
        yield
        torch.cuda.synchronize()
        print(f'[kfac-sync] {name} ok', file=sys.stderr, flush=True)
        return
    if timer is None or (
        torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    ):
        yield
    else:
        with timer.phase(name):
            yield
