"""Gradient-preconditioning epilogues and the device-side KL clip (K-HIP-7).

The GEMM chain ``QG^T [Wg | bg] QA -> scale -> QG (.) QA^T`` runs on
hipBLASLt through ``torch.mm(..., out=)`` into per-layer persistent buffers
(plain library GEMMs); everything between and after the GEMMs is a native
kernel here, so a K-FAC step performs no host synchronisation:

* ``eigen_scale_(v, dgda=..)`` / ``(v, dg=.., da=.., damping=..)``:
  ``v *= dgda`` or ``v /= outer(dg, da) + damping`` in place.
* ``kl_dot_(p, wgrad, bgrad, acc)``: ``acc += <P, [Wg | bg]>`` (fp64 device
  accumulator).
* ``kl_finalize(acc, scale, kl_clip, lr)``: ``scale = min(1,
  sqrt(kl_clip / |acc * lr^2|))`` (1 if acc == 0), resets ``acc``.
* ``apply_grad_(p, wgrad, bgrad, scale)``: ``Wg = s*P[:, :-1]``,
  ``bg = s*P[:, -1]`` written in place into the parameters' ``.grad``.
"""
from __future__ import annotations

import math

import torch

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native


def eigen_scale_(
    v: torch.Tensor,
    *,
    dgda: torch.Tensor | None = None,
    dg: torch.Tensor | None = None,
    da: torch.Tensor | None = None,
    damping: float = 0.0,
) -> torch.Tensor:
    if (
        use_native(v)
        and v.dtype == torch.float32
        and v.stride(1) == 1
        and (dgda is None or dgda.dtype == torch.float32)
        and (dg is None or dg.dtype == torch.float32)
        and (da is None or da.dtype == torch.float32)
    ):
        native().eigen_scale(
            v,
            None if dgda is None else dgda.contiguous(),
            None if dg is None else dg.contiguous(),
            None if da is None else da.contiguous(),
            float(damping),
        )
        return v
    if dgda is not None:
        return v.mul_(dgda)
    assert dg is not None and da is not None
    return v.div_(torch.outer(dg, da) + damping)


def _combined(wgrad: torch.Tensor, bgrad: torch.Tensor | None) -> torch.Tensor:
    w = wgrad.reshape(wgrad.shape[0], -1)
    if bgrad is None:
        return w
    return torch.cat([w, bgrad.reshape(-1, 1)], dim=1)


def _native_ok(p: torch.Tensor, *grads: torch.Tensor | None) -> bool:
    return (
        p.dtype == torch.float32
        and p.stride(1) == 1
        and all(g is None or g.is_contiguous() for g in grads)
        and all(
            g is None
            or g.dtype in (torch.float32, torch.bfloat16, torch.float16)
            for g in grads
        )
    )


def kl_dot_(
    p: torch.Tensor,
    wgrad: torch.Tensor,
    bgrad: torch.Tensor | None,
    acc: torch.Tensor,
) -> None:
    """``acc += sum(P * [Wg | bg])`` with ``acc`` a 1-element fp64 tensor."""
    if use_native(p) and _native_ok(p, wgrad, bgrad):
        native().kl_dot(p, wgrad, bgrad, acc)
        return
    g = _combined(wgrad, bgrad).to(torch.float64)
    acc += (p.to(torch.float64) * g).sum()


def kl_finalize(
    acc: torch.Tensor,
    scale: torch.Tensor,
    kl_clip: float,
    lr: float,
) -> None:
    """Turn the accumulated ``<P, grad>`` into the KL-clip scale, in place."""
    if use_native(acc):
        native().kl_finalize(acc, scale, float(kl_clip), float(lr))
        return
    vg = float(acc.item()) * lr * lr
    s = 1.0 if vg == 0.0 else min(1.0, math.sqrt(kl_clip / abs(vg)))
    scale.fill_(s)
    acc.zero_()


def apply_grad_(
    p: torch.Tensor,
    wgrad: torch.Tensor,
    bgrad: torch.Tensor | None,
    scale: torch.Tensor | float | None,
) -> None:
    """Write ``scale * P`` into the weight / bias gradients in place."""
    if (
        use_native(p)
        and _native_ok(p, wgrad, bgrad)
        and (scale is None or isinstance(scale, torch.Tensor))
    ):
        native().apply_grad(p, wgrad, bgrad, scale)
        return
    rows = wgrad.shape[0]
    src = p
    if scale is not None:
        src = p * scale
    if bgrad is not None:
        wgrad.copy_(src[:, :-1].reshape(wgrad.shape))
        bgrad.copy_(src[:, -1].reshape(bgrad.shape))
    else:
        wgrad.copy_(src.reshape(rows, -1).reshape(wgrad.shape))


class MultiLayerApply:
    """KL clip + gradient write for all layers in three native launches.

    Caches the device descriptor table while the layers' preconditioned
    gradient buffers and parameter gradients keep their storage (the normal
    case: persistent buffers, ``zero_grad(set_to_none=False)`` or DDP bucket
    views).  ``run`` returns False when the fast path does not apply (CPU,
    non-fp32 P, a gradient view that is not in place) so the caller can fall
    back to the per-layer path.
    """

    def __init__(self) -> None:
        self._key: tuple | None = None
        self._table: torch.Tensor | None = None
        self._blocks = 0
        self._acc: torch.Tensor | None = None
        self._scale: torch.Tensor | None = None
        self._params: torch.Tensor | None = None
        self._param_vals: tuple[float, float] | None = None
        self._n = 0

    def _buffers(self, device: torch.device) -> None:
        if self._acc is None or self._acc.device != device:
            self._acc = torch.zeros(1, dtype=torch.float64, device=device)
            self._scale = torch.ones(1, dtype=torch.float32, device=device)
            self._params = torch.zeros(2, dtype=torch.float32, device=device)
            self._param_vals = None

    def prepare(
        self,
        layers: list,
        kl_clip: float | None,
        lr: float,
        use_buffers: bool = False,
    ) -> bool:
        """Build / refresh the descriptor table and the (kl_clip, lr) device
        params.  ``use_buffers`` describes P by each layer's persistent grad
        buffer instead of its current ``grad`` (for graph capture, where P
        is produced inside the graph)."""
        lib = native()
        if lib is None or not layers:
            return False
        ps, ws, bs = [], [], []
        key = []
        for layer in layers:
            p = layer._grad_buf if use_buffers else layer.grad
            if p is None:
                if use_buffers:
                    return False
                raise AssertionError('layer gradient has not been preconditioned')
            if not p.is_cuda or p.dtype != torch.float32 or p.stride(1) != 1:
                return False
            helper = layer.module
            wg = helper.get_weight_grad()
            wm = helper.weight_grad_matrix()
            if not (wm.is_contiguous() and wm.data_ptr() == wg.data_ptr()):
                return False
            if wm.dtype not in (torch.float32, torch.bfloat16, torch.float16):
                return False
            bg = helper.get_bias_grad() if helper.has_bias() else None
            if bg is not None and not bg.is_contiguous():
                return False
            ps.append(p)
            ws.append(wm)
            bs.append(bg)
            key.append((
                p.data_ptr(), tuple(p.shape), p.stride(0), wm.data_ptr(),
                tuple(wm.shape), wm.dtype, None if bg is None else bg.data_ptr(),
                None if bg is None else bg.dtype,
            ))
        key_t = tuple(key)
        if key_t != self._key:
            self._table, self._blocks = lib.build_layer_table(ps, ws, bs)
            self._key = key_t
        self._n = len(ps)
        self._buffers(ps[0].device)
        if kl_clip is not None:
            vals = (float(kl_clip), float(lr))
            if vals != self._param_vals:
                self._params[0].fill_(vals[0])
                self._params[1].fill_(vals[1])
                self._param_vals = vals
        return True

    def launch(self, with_kl: bool) -> None:
        """The three (or one, without KL clip) multi-tensor launches."""
        lib = native()
        if not with_kl:
            lib.apply_multi(self._table, self._n, self._blocks, None)
            return
        lib.kl_dot_multi(self._table, self._n, self._blocks, self._acc)
        lib.kl_finalize_dev(self._acc, self._params, self._scale)
        lib.apply_multi(self._table, self._n, self._blocks, self._scale)

    def run(self, layers: list, kl_clip: float | None, lr: float) -> bool:
        """prepare + launch for an eagerly preconditioned step."""
        if not self.prepare(layers, kl_clip, lr):
            return False
        self.launch(kl_clip is not None)
        for layer in layers:
            layer.grad = None
        return True
