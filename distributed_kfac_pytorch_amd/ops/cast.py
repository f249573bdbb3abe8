"""Fused autocast weight casts (csrc/cast.hip).

Under ``torch.autocast(dtype=torch.bfloat16)`` PyTorch casts every conv /
linear weight to bf16 on its own at each forward, and every bf16 weight
gradient back to fp32 on its own at each backward: 57 + 56 tiny kernels per
ResNet-50 step, ~0.55 ms of a ~8.6 ms graph-replayed SGD step on MI355X.
``enable_fused_weight_cast(model)`` produces the same bf16 copies (same
round-to-nearest-even rounding, same strides) with one multi-tensor launch
per parameter group, and their gradients back to fp32 with one launch per
group, through an autograd function -- the parameters, their fp32
``.grad`` and every hook (K-FAC's module hooks, DDP's gradient hooks) are
unchanged.

Groups follow the backward order in ~``group_mb`` chunks (DDP's default
bucket size), so a group's gradients are released as soon as its last
weight gradient exists and DDP still overlaps its all-reduces with the rest
of the backward pass.

On CPU, without the native extension, or outside a matching autocast region
the modules run their plain forward (autocast's own casts).
"""
from __future__ import annotations

from typing import Any

import torch
from torch import nn

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops.precondition import _TableCache
from distributed_kfac_pytorch_amd.ops.precondition import _used_here

_ALIGN = 8  # elements: 16-B aligned bf16 segments, 32-B fp32


def _ru(x: int, a: int) -> int:
    return (x + a - 1) // a * a


class _Caster:
    """Cast lists of dense tensors with one launch, outputs packed in one
    buffer (each output keeps its source's shape and strides)."""

    def __init__(self) -> None:
        # one entry per parameter group and direction: a whole-step capture of
        # both step kinds builds ~20 tables, and pinned staging cannot be
        # allocated while a capture runs, so keep ample spare slots
        self._cache = _TableCache(size=64)

    def cast(self, srcs: list[torch.Tensor], dtype: torch.dtype) -> list[torch.Tensor]:
        lib = native()
        total = sum(_ru(s.numel(), _ALIGN) for s in srcs)
        flat = torch.empty(max(total, 1), dtype=dtype, device=srcs[0].device)
        outs, off = [], 0
        for s in srcs:
            outs.append(flat.as_strided(s.shape, s.stride(), off))
            off += _ru(s.numel(), _ALIGN)
        if lib is None or not flat.is_cuda:
            for o, s in zip(outs, srcs):  # reference path (CPU tests)
                o.copy_(s)
            return outs
        key = (dtype, flat.data_ptr()) + tuple((s.data_ptr(), s.numel()) for s in srcs)
        ent = self._cache.get(key)
        if ent is None:
            slots = self._cache.reserve()
            tab, blocks, host = lib.build_cast_table(srcs, outs, slots[0])
            ent = self._cache.put(key, (tab, blocks, host), slots)
        tab, blocks, _ = ent
        lib.cast_multi(_used_here(tab), len(srcs), blocks, dtype == torch.bfloat16)
        return outs


_CASTER: _Caster | None = None


def _caster() -> _Caster:
    global _CASTER
    if _CASTER is None:
        _CASTER = _Caster()
    return _CASTER


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense in some dimension order (the storage span
    equals numel), e.g. contiguous or channels_last."""
    expected = 1
    for d in sorted(range(t.dim()), key=lambda d: (t.stride(d), t.shape[d])):
        if t.shape[d] == 1:
            continue
        if t.stride(d) != expected:
            return False
        expected *= t.shape[d]
    return True


class _FusedCast(torch.autograd.Function):
    @staticmethod
    def forward(ctx: Any, dtype: torch.dtype, *ws: torch.Tensor) -> tuple[torch.Tensor, ...]:
        ctx.src_dtype = ws[0].dtype
        ctx.meta = [(w.shape, w.stride()) for w in ws]
        return tuple(_caster().cast(list(ws), dtype))

    @staticmethod
    def backward(ctx: Any, *gs: torch.Tensor | None) -> tuple[Any, ...]:
        idx, srcs = [], []
        for i, (g, (shape, stride)) in enumerate(zip(gs, ctx.meta)):
            if g is None:
                continue
            if g.stride() != stride or not _dense(g):
                # the cast runs in storage order: match the weight's layout
                g = torch.empty_strided(shape, stride, dtype=g.dtype, device=g.device).copy_(g)
            idx.append(i)
            srcs.append(g)
        out: list[torch.Tensor | None] = [None] * len(gs)
        if srcs:
            for i, r in zip(idx, _caster().cast(srcs, ctx.src_dtype)):
                out[i] = r
        return (None, *out)


def _copies(self: nn.Module) -> dict | None:
    """This forward's fused bf16 copies, only inside the autocast region
    they were made for (a call outside it runs the plain forward)."""
    c = self.__dict__.get('_fused_cast')
    if c is None or 'weight' not in c:
        return None
    dt = c['device_type']
    if not torch.is_autocast_enabled(dt) or torch.get_autocast_dtype(dt) != c['dtype']:
        return None
    return c


def _conv_forward(self: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    c = _copies(self)
    if c is None:
        return nn.Conv2d.forward(self, x)
    return self._conv_forward(x, c['weight'], c.get('bias'))


def _linear_forward(self: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    c = _copies(self)
    if c is None:
        return nn.Linear.forward(self, x)
    return torch.nn.functional.linear(x, c['weight'], c.get('bias'))


class FusedWeightCast:
    """Handle returned by ``enable_fused_weight_cast`` (``remove()`` undoes
    it)."""

    def __init__(self, model: nn.Module, dtype: torch.dtype, group_mb: float,
                 device_type: str = 'cuda') -> None:
        self.model = model
        self.dtype = dtype
        self.device_type = device_type
        self.mods: list[nn.Module] = []
        for m in model.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)) and m.weight.dtype == torch.float32:
                self.mods.append(m)
        for m in self.mods:
            m.forward = (_conv_forward if isinstance(m, nn.Conv2d) else _linear_forward).__get__(m)
        # parameter groups in backward (reverse registration) order
        cap = int(group_mb * (1 << 20))
        self.groups: list[list[tuple[nn.Module, str]]] = []
        cur: list[tuple[nn.Module, str]] = []
        size = 0
        for m in reversed(self.mods):
            for name in ('weight', 'bias'):
                p = getattr(m, name, None)
                if p is None:
                    continue
                cur.append((m, name))
                size += p.numel() * p.element_size()
            if size >= cap:
                self.groups.append(cur)
                cur, size = [], 0
        if cur:
            self.groups.append(cur)
        self._pre = model.register_forward_pre_hook(self._before)
        self._post = model.register_forward_hook(self._after)

    def _active(self) -> bool:
        if not self.mods or self.mods[0].weight.device.type != self.device_type:
            return False
        if self.device_type == 'cuda' and native() is None:
            return False
        return (torch.is_autocast_enabled(self.device_type)
                and torch.get_autocast_dtype(self.device_type) == self.dtype)

    def _before(self, module: nn.Module, args: Any) -> None:
        # copies left behind by a forward that raised (e.g. OOM) must never
        # be used by a later forward
        for m in self.mods:
            m.__dict__.pop('_fused_cast', None)
        if not self._active():
            return
        for group in self.groups:
            ps = [getattr(m, n) for m, n in group]
            if not all(_dense(p) for p in ps):
                continue
            outs = _FusedCast.apply(self.dtype, *ps)
            for (m, n), o in zip(group, outs):
                c = m.__dict__.setdefault('_fused_cast', {'device_type': self.device_type,
                                                          'dtype': self.dtype})
                c[n] = o

    def _after(self, module: nn.Module, args: Any, output: Any) -> None:
        for m in self.mods:
            m.__dict__.pop('_fused_cast', None)

    def remove(self) -> None:
        self._pre.remove()
        self._post.remove()
        for m in self.mods:
            m.__dict__.pop('forward', None)
            m.__dict__.pop('_fused_cast', None)


def enable_fused_weight_cast(model: nn.Module, dtype: torch.dtype = torch.bfloat16,
                             group_mb: float = 25.0, device_type: str = 'cuda') -> FusedWeightCast:
    """Cast the model's conv / linear weights (and biases) to ``dtype`` with
    fused multi-tensor launches whenever its forward runs under an autocast
    region of that dtype on ``device_type`` (``'cpu'``: the same logic with
    per-tensor copies, for tests).  Returns a handle with ``remove()``."""
    return FusedWeightCast(model, dtype, group_mb, device_type)
