"""Registration of model modules as K-FAC layers
(reference ``kfac/layers/register.py:1-94``).

Leaf modules are walked in ``named_modules`` order; a module is registered
when no ``skip_layers`` regex ``re.search``-matches its name or class name,
every parameter requires grad, and a helper exists for its type.  Supported
types: ``nn.Linear`` (and subclasses, e.g. the tensor-parallel linears) and
``nn.Conv2d`` with dilation 1 / groups 1 / zero padding.  Grouped or dilated
convolutions are skipped with a warning (the reference registers them and
then computes wrong shapes).  ``nn.Embedding`` is handled by
``layers.embedding`` when the preconditioner enables it.
"""
from __future__ import annotations

import re
import warnings
from typing import Any

import torch

from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.layers.modules import Conv2dModuleHelper
from distributed_kfac_pytorch_amd.layers.modules import LinearModuleHelper
from distributed_kfac_pytorch_amd.layers.modules import ModuleHelper

KNOWN_MODULES = {'linear', 'conv2d'}
LINEAR_TYPES: tuple[type[torch.nn.Module], ...] = (torch.nn.Linear,)
CONV2D_TYPES: tuple[type[torch.nn.Module], ...] = (torch.nn.Conv2d,)


def get_flattened_modules(
    root: torch.nn.Module,
) -> list[tuple[str, torch.nn.Module]]:
    """``(name, module)`` for every leaf (childless) module of ``root``."""
    return [
        (name, mod)
        for name, mod in root.named_modules()
        if next(mod.children(), None) is None
    ]


def requires_grad(module: torch.nn.Module) -> bool:
    """False if any parameter of ``module`` has ``requires_grad=False``."""
    return all(p.requires_grad for p in module.parameters())


def get_module_helper(module: torch.nn.Module) -> ModuleHelper | None:
    """Helper wrapping ``module``, or None if the type is unsupported."""
    if isinstance(module, LINEAR_TYPES):
        return LinearModuleHelper(module)
    if isinstance(module, CONV2D_TYPES):
        try:
            return Conv2dModuleHelper(module)
        except ValueError as e:
            warnings.warn(f'not registering {module!r} with K-FAC: {e}')
            return None
    return None


def any_match(query: str, patterns: list[str]) -> bool:
    """True if any regex in ``patterns`` is found anywhere in ``query``."""
    return any(re.search(p, query) is not None for p in patterns)


def register_modules(
    model: torch.nn.Module,
    kfac_layer_type: type[KFACBaseLayer],
    skip_layers: list[str],
    helper_factory: Any = None,
    **layer_kwargs: Any,
) -> dict[torch.nn.Module, tuple[str, KFACBaseLayer]]:
    """Map each supported module of ``model`` to ``(name, K-FAC layer)``.

    Args:
        model: model to scan.
        kfac_layer_type: layer class to instantiate.
        skip_layers: regexes matched against module names and class names.
        helper_factory: optional ``module -> ModuleHelper | None`` overriding
            ``get_module_helper`` (used by the embedding / TP paths).
        **layer_kwargs: forwarded to ``kfac_layer_type``.
    """
    factory = helper_factory or get_module_helper
    layers: dict[torch.nn.Module, tuple[str, KFACBaseLayer]] = {}
    for name, module in get_flattened_modules(model):
        if any_match(name, skip_layers):
            continue
        if any_match(module.__class__.__name__, skip_layers):
            continue
        if not requires_grad(module):
            continue
        helper = factory(module)
        if helper is None:
            continue
        assert module not in layers
        layers[module] = (name, kfac_layer_type(helper, **layer_kwargs))
    return layers
