"""Damped-inverse K-FAC layer (reference ``kfac/layers/inverse.py:19-233``).

    A_inv = (A + damping I)^-1,  G_inv = (G + damping I)^-1  (fp32)
    P     = G_inv [Wg | bg] A_inv

The damped factors are SPD, so the inverse is a Cholesky factorisation plus
``cholesky_inverse`` (``ops.linalg.damped_inverse``) instead of an LU
inverse; non-symmetric factors (a test-only case in the reference) use
``torch.linalg.inv``.  Inverses are symmetric, so ``symmetry_aware``
broadcasts send only the upper triangle (native pack/unpack kernels).
"""
from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.layers.base import _nbytes
from distributed_kfac_pytorch_amd.layers.base import _resolve
from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.ops import linalg
from distributed_kfac_pytorch_amd.parallel.comm import FutureType
from distributed_kfac_pytorch_amd.parallel.comm import get_rank


class KFACInverseLayer(KFACBaseLayer):
    """K-FAC layer preconditioning with explicit damped inverses."""

    def __init__(self, module: Any, **kwargs: Any) -> None:
        super().__init__(module, **kwargs)
        self._a_inv: torch.Tensor | FutureType | None = None
        self._g_inv: torch.Tensor | FutureType | None = None
        self._tmp1: torch.Tensor | None = None

    @property
    def a_inv(self) -> torch.Tensor | None:
        self._a_inv = _resolve(self._a_inv)
        return self._a_inv

    @a_inv.setter
    def a_inv(self, v: torch.Tensor | FutureType | None) -> None:
        self._a_inv = v

    @property
    def g_inv(self) -> torch.Tensor | None:
        self._g_inv = _resolve(self._g_inv)
        return self._g_inv

    @g_inv.setter
    def g_inv(self, v: torch.Tensor | FutureType | None) -> None:
        self._g_inv = v

    def memory_usage(self) -> dict[str, int]:
        sizes = super().memory_usage()
        sizes['a_inverses'] = _nbytes(self.a_inv)
        sizes['g_inverses'] = _nbytes(self.g_inv)
        return sizes

    def _sym(self) -> bool:
        return self.symmetric_factors and self.symmetry_aware

    def _bcast(self, t: torch.Tensor, src: int, group: dist.ProcessGroup | None,
               bucketed: bool) -> Any:
        if self._sym():
            # triangle-packed broadcasts stay per tensor
            return self.tdc.broadcast(t, src=src, group=group, symmetric=True)
        if bucketed and self.tdc.bucket_cap_bytes > 0 and t.is_contiguous():
            return self.tdc.broadcast_bucketed(t, src=src, group=group)
        return self.tdc.broadcast(t, src=src, group=group)

    def broadcast_a_inv(self, src: int, group: dist.ProcessGroup | None = None,
                        bucketed: bool = False) -> None:
        if self.a_inv is None:
            if get_rank() == src:
                raise RuntimeError(
                    f'Attempt to broadcast A inv from src={src} but this rank '
                    'has not computed A inv yet.',
                )
            d = self.module.a_factor_shape[0]
            self.a_inv = torch.empty(
                d, d, device=self.module.device, dtype=self.inv_dtype,
            )
        self.a_inv = self._bcast(self.a_inv, src, group, bucketed)

    def broadcast_g_inv(self, src: int, group: dist.ProcessGroup | None = None,
                        bucketed: bool = False) -> None:
        if self.g_inv is None:
            if get_rank() == src:
                raise RuntimeError(
                    f'Attempt to broadcast G inv from src={src} but this rank '
                    'has not computed G inv yet.',
                )
            d = self.module.g_factor_shape[0]
            self.g_inv = torch.empty(
                d, d, device=self.module.device, dtype=self.inv_dtype,
            )
        self.g_inv = self._bcast(self.g_inv, src, group, bucketed)

    def _inverse(self, f: torch.Tensor, damping: float) -> torch.Tensor:
        if self.symmetric_factors:
            return linalg.damped_inverse(f, damping).to(self.inv_dtype)
        d = torch.eye(f.shape[0], dtype=f.dtype, device=f.device) * damping
        return torch.linalg.inv((f + d).to(torch.float32)).to(self.inv_dtype)

    @staticmethod
    def _install(old: Any, new: torch.Tensor) -> torch.Tensor:
        """Copy ``new`` into the existing inverse buffer when possible, so
        A^-1 / G^-1 keep one device address across inverse updates: the
        grouped-GEMM descriptor tables and captured HIP graphs
        (``StepGraphs``, ``graphs.GraphedTrainStep``) hold that address."""
        if (
            isinstance(old, torch.Tensor)
            and old.shape == new.shape
            and old.dtype == new.dtype
            and old.device == new.device
            and old.is_contiguous()
        ):
            if old.data_ptr() != new.data_ptr():
                old.copy_(new)
            return old
        return new.contiguous()

    def set_a_inv(self, inv: torch.Tensor) -> None:
        self.a_inv = self._install(self.a_inv, inv.to(self.inv_dtype))

    def set_g_inv(self, inv: torch.Tensor) -> None:
        self.g_inv = self._install(self.g_inv, inv.to(self.inv_dtype))

    def compute_a_inv(self, damping: float = 0.001) -> None:
        if self.a_factor is None:
            raise RuntimeError('Cannot invert A before A has been computed')
        self.set_a_inv(self._inverse(self.a_factor, damping))

    def compute_g_inv(self, damping: float = 0.001) -> None:
        if self.g_factor is None:
            raise RuntimeError('Cannot invert G before G has been computed')
        self.set_g_inv(self._inverse(self.g_factor, damping))

    def preconditioned_grad(self, damping: float = 0.001) -> None:
        """P = G_inv [Wg | bg] A_inv into the persistent grad buffer."""
        a_inv, g_inv = self.a_inv, self.g_inv
        if a_inv is None or g_inv is None:
            raise RuntimeError(
                'Cannot precondition gradient before A and G have been '
                'inverted',
            )
        dt = a_inv.dtype
        wg, bg, _ = self.precond_operands()
        wg = wg.to(dt)
        dev = a_inv.device
        shape = (g_inv.shape[0], a_inv.shape[0])
        if self._tmp1 is None or tuple(self._tmp1.shape) != shape or self._tmp1.dtype != dt:
            self._tmp1 = torch.empty(shape, dtype=dt, device=dev)
        t1 = self._tmp1
        # t1 = [Wg | bg] A_inv  without concatenation
        if bg is not None:
            torch.mm(wg, a_inv[:-1], out=t1)
            t1.addr_(bg.reshape(-1).to(dt), a_inv[-1])
        else:
            torch.mm(wg, a_inv, out=t1)
        if dt == torch.float32:
            out = self.precond_out(dev)
            torch.mm(g_inv, t1, out=out)
        else:
            out = (g_inv @ t1).to(torch.float32)
        self.grad = out
