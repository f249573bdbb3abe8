"""Loader for the in-tree HIP extension (``distributed_kfac_pytorch_amd._C``).

Policy:
* GPU tensors go through the native gfx950 kernels.  If the extension is
  missing on a GPU box the op RAISES (no silent eager fallback) unless
  ``KFAC_ALLOW_TORCH_FALLBACK=1`` is set (used only for A/B benchmarking of
  the reference math against the kernels).
* CPU tensors use the PyTorch reference math in the op modules (the
  multi-process gloo tests run there).
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType

import torch

_lib: ModuleType | None = None
_err: BaseException | None = None
_tried = False


def _load() -> None:
    global _lib, _err, _tried
    if _tried:
        return
    _tried = True
    if os.environ.get('KFAC_DISABLE_NATIVE') == '1':
        _err = RuntimeError('native kernels disabled by KFAC_DISABLE_NATIVE=1')
        return
    try:
        _lib = importlib.import_module('distributed_kfac_pytorch_amd._C')
    except BaseException as e:  # noqa: BLE001 - reported on first GPU use
        _err = e


def native() -> ModuleType | None:
    """The extension module, or None if it is not built / disabled."""
    _load()
    return _lib


def available() -> bool:
    return native() is not None


def load_error() -> BaseException | None:
    _load()
    return _err


def fallback_allowed() -> bool:
    return os.environ.get('KFAC_ALLOW_TORCH_FALLBACK') == '1'


def use_native(*tensors: torch.Tensor) -> bool:
    """True if this call must run the HIP kernels.

    Raises when the tensors live on the GPU but the extension is unusable and
    the torch fallback was not explicitly allowed.
    """
    if not any(t.is_cuda for t in tensors):
        return False
    if native() is not None:
        return True
    if fallback_allowed() or os.environ.get('KFAC_DISABLE_NATIVE') == '1':
        return False
    raise RuntimeError(
        'distributed_kfac_pytorch_amd native HIP extension is not available '
        f'({_err!r}); build it with `python tools/build_native.py` or set '
        'KFAC_ALLOW_TORCH_FALLBACK=1 to run the PyTorch reference math.',
    )


def flush_table_uploads() -> int:
    """Upload the descriptor tables built inside the HIP-graph capture that
    just ended (csrc/bindings.cpp ``upload_table``: captures record no copy
    node; the tables are uploaded once, eagerly, before the first replay).
    Every site that captures a graph calls this right after the capture."""
    lib = native()
    return int(lib.flush_table_uploads()) if lib is not None else 0
