"""Per-layer K-FAC state machine (reference ``kfac/layers/base.py:18-422``).

One ``KFACBaseLayer`` per registered module holds the batch accumulators,
the running factors, the second-order state (in subclasses) and the
preconditioned gradient, and exposes the stages the preconditioner drives:
save -> update -> reduce -> compute -> broadcast -> precondition -> update.

MI355X-specific behaviour:

* ``save_layer_input`` does not clone the activation (reference
  ``base.py:346-349``): the SYRK that consumes it is enqueued on the same
  HIP stream inside the hook, so stream order guarantees it reads the value
  before any later in-place op rewrites it.
* ``save_and_update_a`` / ``save_and_update_g`` fuse accumulation, the
  1/count average, identity initialisation and the EMA into one SYRK launch
  (``C = decay*C + (1-decay)*scale*X^T X``) when there is exactly one
  micro-batch per update (the common case); the generic path keeps the
  reference's accumulate-then-update semantics.
* Factors, eigen/inverse state and the preconditioned gradient are updated
  IN PLACE in persistent buffers; collectives return ``AsyncTensor`` handles
  that resolve lazily through the properties, like the reference's futures.
"""
from __future__ import annotations


from typing import Callable

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.enums import AllreduceMethod
from distributed_kfac_pytorch_amd.layers.modules import ModuleHelper
from distributed_kfac_pytorch_amd.ops import comm_pack
from distributed_kfac_pytorch_amd.ops import factors as factor_ops
from distributed_kfac_pytorch_amd.parallel.comm import AsyncTensor
from distributed_kfac_pytorch_amd.parallel.comm import Future
from distributed_kfac_pytorch_amd.parallel.comm import FutureType
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size
from distributed_kfac_pytorch_amd.parallel.comm import (
    TorchDistributedCommunicator,
)
from distributed_kfac_pytorch_amd.utils.env import getenv


def _resolve(value: torch.Tensor | FutureType | None) -> torch.Tensor | None:
    if isinstance(value, Future):
        return value.wait()
    return value


def _nbytes(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.nelement() * t.element_size()


class KFACBaseLayer:
    """Base K-FAC layer: factor accumulation, reduction, gradient handling."""

    def __init__(
        self,
        module: ModuleHelper,
        *,
        tdc: TorchDistributedCommunicator,
        allreduce_method: AllreduceMethod = AllreduceMethod.ALLREDUCE,
        factor_dtype: torch.dtype | None = None,
        grad_scaler: (
            torch.cuda.amp.GradScaler | Callable[[], float] | None
        ) = None,
        inv_dtype: torch.dtype = torch.float32,
        symmetry_aware: bool = False,
    ) -> None:
        """Init KFACBaseLayer.

        Args:
            module (ModuleHelper): helper wrapping the torch module.
            tdc (TorchDistributedCommunicator): shared communicator.
            allreduce_method (AllreduceMethod): plain or bucketed factor
                all-reduce.
            factor_dtype (torch.dtype): storage dtype of the factors.  None
                keeps fp32 for half-precision activations (the MFMA
                accumulator precision) and the activation dtype otherwise.
            grad_scaler: AMP GradScaler (or callable returning the scale);
                G contributions are unscaled by it.
            inv_dtype (torch.dtype): dtype of eigenbases / inverses.
            symmetry_aware (bool): communicate only upper triangles.
        """
        self.module = module
        self.tdc = tdc
        self.allreduce_method = allreduce_method
        self.factor_dtype = factor_dtype
        # a GradScaler's scale tensor lives on the device: the G unscale
        # 1/s^2 is computed and applied there (no host sync per layer)
        self._scaler = grad_scaler if isinstance(grad_scaler, torch.amp.GradScaler) else None
        if isinstance(grad_scaler, torch.amp.GradScaler):
            grad_scaler = grad_scaler.get_scale
        self.grad_scaler: Callable[[], float] | None = grad_scaler
        self.inv_dtype = inv_dtype
        self.symmetry_aware = symmetry_aware
        self.eps = 1e-10
        self.symmetric_factors = self.module.has_symmetric_factors()

        self._a_batch: torch.Tensor | None = None
        self._g_batch: torch.Tensor | None = None
        self._a_count: int = 0
        self._g_count: int = 0
        self._a_factor: torch.Tensor | FutureType | None = None
        self._g_factor: torch.Tensor | FutureType | None = None
        # packed all-reduce home of each factor (parallel/comm.py
        # PackedFactorBuffer): (buffer, key, world) once registered; `live`
        # while the packed triangle, not the dense tensor, is authoritative
        self._homes: dict[str, tuple | None] = {'A': None, 'G': None}
        self._live: dict[str, bool] = {'A': False, 'G': False}
        self._dense: dict[str, torch.Tensor | None] = {'A': None, 'G': None}
        self._grad: torch.Tensor | FutureType | None = None
        # persistent output buffer of preconditioned_grad / broadcast_grad
        self._grad_buf: torch.Tensor | None = None

    def __repr__(self) -> str:
        return f'{self.__class__.__name__}({self.module!r})'

    # ------------------------------------------------------------ properties
    @property
    def a_factor(self) -> torch.Tensor | None:
        self._a_factor = _resolve(self._a_factor)
        return self._a_factor

    @a_factor.setter
    def a_factor(self, value: torch.Tensor | FutureType | None) -> None:
        self._a_factor = value
        self._live['A'] = False

    @property
    def g_factor(self) -> torch.Tensor | None:
        self._g_factor = _resolve(self._g_factor)
        return self._g_factor

    @g_factor.setter
    def g_factor(self, value: torch.Tensor | FutureType | None) -> None:
        self._g_factor = value
        self._live['G'] = False

    @property
    def grad(self) -> torch.Tensor | None:
        self._grad = _resolve(self._grad)
        return self._grad

    @grad.setter
    def grad(self, value: torch.Tensor | FutureType | None) -> None:
        self._grad = value

    # ------------------------------------------------------------ checkpoint
    def _a_to_ref(self, a: torch.Tensor) -> torch.Tensor:
        conv = getattr(self.module, 'a_to_reference_order', None)
        return conv(a) if conv is not None else a

    def _a_from_ref(self, a: torch.Tensor) -> torch.Tensor:
        conv = getattr(self.module, 'a_from_reference_order', None)
        return conv(a) if conv is not None else a

    def state_dict(self) -> dict[str, torch.Tensor | None]:
        """``{'A': factor, 'G': factor}`` in reference column order.

        Tensors are snapshots (the live factors are updated in place).
        """
        a, g = self.a_factor, self.g_factor
        return {
            'A': None if a is None else self._a_to_ref(a).clone(),
            'G': None if g is None else g.clone(),
        }

    def load_state_dict(self, state_dict: dict[str, torch.Tensor | None]) -> None:
        """Load factors (moved to the module's device)."""
        if 'A' not in state_dict or 'G' not in state_dict:
            raise KeyError("KFACLayer state_dict must contain keys 'A' and 'G'")
        device = self.module.device
        a, g = state_dict['A'], state_dict['G']
        if a is not None:
            self.a_factor = self._a_from_ref(a.to(device)).contiguous()
        if g is not None:
            self.g_factor = g.to(device).contiguous()

    def memory_usage(self) -> dict[str, int]:
        return {
            'a_factors': _nbytes(self.a_factor),
            'g_factors': _nbytes(self.g_factor),
            'a_batch': _nbytes(self._a_batch),
            'g_batch': _nbytes(self._g_batch),
        }

    # ---------------------------------------------------------- second order
    def broadcast_a_inv(self, src: int, group: dist.ProcessGroup | None = None,
                        bucketed: bool = False) -> None:
        raise NotImplementedError

    def broadcast_g_inv(self, src: int, group: dist.ProcessGroup | None = None,
                        bucketed: bool = False) -> None:
        raise NotImplementedError

    def compute_a_inv(self, damping: float = 0.001) -> None:
        raise NotImplementedError

    def compute_g_inv(self, damping: float = 0.001) -> None:
        raise NotImplementedError

    def preconditioned_grad(self, damping: float = 0.001) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------- gradients
    def grad_shape(self) -> tuple[int, int]:
        g = self.module.g_factor_shape[0]
        return (g, self.module.a_factor_shape[0])

    def _grad_buffer(self, device: torch.device) -> torch.Tensor:
        shape = self.grad_shape()
        if (
            self._grad_buf is None
            or tuple(self._grad_buf.shape) != shape
            or self._grad_buf.device != device
        ):
            self._grad_buf = torch.empty(shape, dtype=torch.float32, device=device)
        return self._grad_buf

    def precond_operands(self) -> tuple[torch.Tensor, torch.Tensor | None, bool]:
        """``(Wg matrix, bias grad or None, stable)`` that preconditioning
        reads.  ``stable``: the matrix is the parameter gradient itself (not
        a reshaped copy), so its address is fixed between steps and the
        grouped GEMM tables keyed on it stay valid.  Tensor-parallel layers
        return their gathered full-gradient buffers instead."""
        helper = self.module
        wg = helper.get_weight_grad()
        wm = helper.weight_grad_matrix()
        bg = helper.get_bias_grad() if helper.has_bias() else None
        stable = wg is not None and wm.is_contiguous() and wm.data_ptr() == wg.data_ptr()
        return wm, bg, stable

    def precond_out(self, device: torch.device) -> torch.Tensor:
        """fp32 buffer receiving the preconditioned gradient P."""
        return self._grad_buffer(device)

    def broadcast_grad(
        self,
        src: int,
        group: dist.ProcessGroup | None = None,
        bucketed: bool = False,
    ) -> None:
        """Broadcast the preconditioned gradient from ``src`` (every rank of
        the receiver group enters).  ``bucketed`` routes it through the
        communicator's fused per-(group, src) broadcast buckets; the caller
        must then call ``tdc.flush_broadcast_buckets()`` on every rank."""
        if self.grad is None:
            if get_rank() == src:
                raise RuntimeError(
                    f'Attempt to broadcast gradient from src={src} but this '
                    'rank has not computed the preconditioned gradient yet.',
                )
            self.grad = self._grad_buffer(self.module.device)
        g = self.grad
        if bucketed and self.tdc.bucket_cap_bytes > 0 and g.is_contiguous():
            # fused per-group exchange (one all-gather of every member's
            # share); flushed by the preconditioner
            self.grad = self.tdc.exchange_bucketed(g, src=src, group=group)
        else:
            self.grad = self.tdc.broadcast(g, src=src, group=group)

    def update_grad(self, scale: torch.Tensor | float | None = None) -> None:
        """Write ``scale * preconditioned grad`` into the module gradients."""
        grad = self.grad
        if grad is None:
            raise RuntimeError(
                'preconditioned gradient is None. This may be because '
                'update_grad() was called before preconditioned_grad()',
            )
        self.module.write_grad(grad, scale)
        self.grad = None

    # --------------------------------------------------------------- factors
    def _allreduce(self):  # noqa: ANN202
        if self.allreduce_method == AllreduceMethod.ALLREDUCE:
            return self.tdc.allreduce
        if self.allreduce_method == AllreduceMethod.ALLREDUCE_BUCKETED:
            return self.tdc.allreduce_bucketed
        raise AssertionError(f'Unknown allreduce_method={self.allreduce_method}')

    def reduce_a_factor(self, group: dist.ProcessGroup | None = None) -> None:
        """Start the (averaging) all-reduce of A; all group ranks enter."""
        if self._packed_reduce('A', group):
            return
        if self.a_factor is None:
            raise RuntimeError('a_factor is None, cannot reduce')
        self.a_factor = self._allreduce()(
            self.a_factor,
            average=True,
            symmetric=self._pack_factors(),
            group=group,
        )

    def reduce_g_factor(self, group: dist.ProcessGroup | None = None) -> None:
        """Start the (averaging) all-reduce of G; all group ranks enter."""
        if self._packed_reduce('G', group):
            return
        if self.g_factor is None:
            raise RuntimeError('g_factor is None, cannot reduce')
        self.g_factor = self._allreduce()(
            self.g_factor,
            average=True,
            symmetric=self._pack_factors(),
            group=group,
        )

    # ------------------------------------------------- packed factor reduce
    def _packed_ok(self, group: dist.ProcessGroup | None) -> bool:
        """The factor all-reduce goes through the persistent packed buffer:
        symmetric factors, more than one rank, fp32, and a GPU
        (``KFAC_PACKED_FACTORS``: auto = GPU only, 1 = also the CPU
        emulation used by the gloo tests, 0 = off).  The slot bookkeeping is
        host-side, so auto stays off under the opt-in multi-rank step graphs
        (``KFAC_STEP_GRAPHS_MULTI=1``), whose replays would skip it."""
        mode = getenv('KFAC_PACKED_FACTORS', 'auto')
        if mode == '0' or not self._pack_factors() or get_world_size(group) == 1:
            return False
        if mode == 'auto' and getenv('KFAC_STEP_GRAPHS_MULTI', '0') == '1':
            return False
        if self.factor_dtype not in (None, torch.float32):
            return False
        return self.module.device.type == 'cuda' or mode == '1'

    def _set_factor(self, which: str, value: torch.Tensor | FutureType | None) -> None:
        # internal assignment that keeps the packed slot authoritative
        if which == 'A':
            self._a_factor = value
        else:
            self._g_factor = value

    def _materialise(self, which: str, buf, key, scale: float) -> torch.Tensor:  # type: ignore[no-untyped-def]
        """Dense factor = scale x the symmetric matrix of the slot (one
        unpack into a persistent buffer)."""
        sl = buf.view(key)
        d = self.module.a_factor_shape[0] if which == 'A' else self.module.g_factor_shape[0]
        dense = self._dense[which]
        if dense is None or dense.shape != (d, d) or dense.device != sl.device:
            dense = torch.empty(d, d, dtype=sl.dtype, device=sl.device)
            self._dense[which] = dense
        comm_pack.triu_unpack_(dense, sl, scale)
        return dense

    def _packed_reduce(self, which: str, group: dist.ProcessGroup | None) -> bool:
        if not self._packed_ok(group):
            return False
        world = get_world_size(group)
        if not self._live[which]:
            # (re-)enter packed mode from the dense local factor: one pack
            dense = self.a_factor if which == 'A' else self.g_factor
            if dense is None:
                raise RuntimeError(f'{which.lower()}_factor is None, cannot reduce')
            if dense.dtype != torch.float32 or dense.dim() != 2:
                return False
            buf = self.tdc.packed_buffer(group, dense.dtype, dense.device)
            key = (id(self), which)
            n = dense.shape[0] * (dense.shape[0] + 1) // 2
            buf.wait(key)
            sl = buf.view(key, n, dense)
            sl.copy_(comm_pack.triu_pack(dense.contiguous()))
            sl.mul_(1.0 / world)
            self._homes[which] = (buf, key, world)
            self._live[which] = True
        buf, key, _ = self._homes[which]  # type: ignore[misc]
        buf.mark(key)
        self._set_factor(which, self.tdc.packed_result(
            buf, key, lambda: self._materialise(which, buf, key, 1.0)))
        return True

    def _packed_update(self, which: str, x: torch.Tensor, alpha: float, beta: float,
                       alpha_scale: torch.Tensor | None = None) -> bool:
        """Fused EMA straight into the packed slot: slot = (beta F_avg +
        alpha X^T X) / world, F_avg the slot's reduced value."""
        home = self._homes[which]
        if home is None or not self._live[which]:
            return False
        buf, key, world = home
        buf.wait(key)
        sl = buf.view(key)
        if which == 'A':
            self.module.accumulate_a_factor(x, sl, alpha / world, beta / world)
        else:
            kw = {} if alpha_scale is None else {'alpha_scale': alpha_scale}
            self.module.accumulate_g_factor(x, sl, alpha / world, beta / world, **kw)
        # the local (not yet reduced) factor, if anything reads it first
        self._set_factor(which, AsyncTensor(
            finalize=lambda: self._materialise(which, buf, key, float(world))))
        return True

    def _pack_factors(self) -> bool:
        """Reduce only the upper triangle of the factors.

        The reference packs only with ``symmetry_aware=True``
        (``kfac/layers/base.py:281-335``).  Here the factors are exactly
        symmetric by construction (the SYRK kernel writes the lower triangle
        as the mirror; the CPU path symmetrises), so reducing the triangle and
        mirroring gives bit-identical results with half the bytes on the
        wire -- done whenever the module's factors are symmetric
        (``KFAC_PACK_FACTORS=0`` restores the reference behaviour).
        """
        if not self.symmetric_factors:
            return False
        if getenv('KFAC_PACK_FACTORS', '1') == '0':
            return self.symmetry_aware
        return True

    def reset_batch(self) -> None:
        self._a_batch = None
        self._a_count = 0
        self._g_batch = None
        self._g_count = 0

    def _storage_dtype(self, x: torch.Tensor) -> torch.dtype:
        if self.factor_dtype is not None:
            return self.factor_dtype
        if x.dtype in (torch.float16, torch.bfloat16):
            return torch.float32
        return x.dtype

    def _g_unscale(self) -> float:
        if self.grad_scaler is None:
            return 1.0
        s = float(self.grad_scaler())
        return 1.0 / (s * s)

    def _g_unscale_parts(self, device: torch.device) -> tuple[float, torch.Tensor | None]:
        """(host factor, device factor) of the G unscale: a GradScaler whose
        scale tensor is on ``device`` gives (1, 1/s^2 computed on the
        device); otherwise the reference's host value (one sync)."""
        sc = self._scaler
        t = getattr(sc, '_scale', None) if sc is not None else None
        if isinstance(t, torch.Tensor) and t.device == device and device.type == 'cuda':
            inv = t.float().reciprocal()
            return 1.0, (inv * inv).reshape(1)
        return self._g_unscale(), None

    def save_layer_input(self, input: list[torch.Tensor]) -> None:
        """Accumulate the A contribution of one forward input."""
        self._save_a(input[0])

    def _save_a(self, a: torch.Tensor) -> None:
        dtype = self._storage_dtype(a)
        d = self.module.a_factor_shape[0]
        if self._a_batch is None:
            self._a_batch = torch.empty(d, d, dtype=dtype, device=a.device)
            self.module.accumulate_a_factor(a, self._a_batch, 1.0, 0.0)
            self._a_count = 1
        else:
            self.module.accumulate_a_factor(a, self._a_batch, 1.0, 1.0)
            self._a_count += 1

    def save_layer_grad_output(self, grad_output: tuple[torch.Tensor, ...]) -> None:
        """Accumulate the G contribution of one output gradient."""
        self._save_g(grad_output[0])

    def _save_g(self, g: torch.Tensor) -> None:
        dtype = self._storage_dtype(g)
        d = self.module.g_factor_shape[0]
        alpha, dev_scale = self._g_unscale_parts(g.device)
        kw = {} if dev_scale is None else {'alpha_scale': dev_scale}
        if self._g_batch is None:
            self._g_batch = torch.empty(d, d, dtype=dtype, device=g.device)
            self.module.accumulate_g_factor(g, self._g_batch, alpha, 0.0, **kw)
            self._g_count = 1
        else:
            self.module.accumulate_g_factor(g, self._g_batch, alpha, 1.0, **kw)
            self._g_count += 1

    @staticmethod
    def _ema_(factor: torch.Tensor, batch: torch.Tensor, alpha: float, count: int) -> None:
        # factor = alpha*factor + (1-alpha)*batch/count
        w = (1.0 - alpha) / count
        if batch.dtype != factor.dtype:
            batch = batch.to(factor.dtype)
        factor.mul_(alpha).add_(batch, alpha=w)

    def _new_identity(self, d: int, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
        out = torch.empty(d, d, dtype=dtype, device=device)
        return factor_ops.identity_(out)

    def update_a_factor(self, alpha: float = 0.95) -> None:
        """Fold the accumulated batch factor into the running average."""
        if self._a_batch is None:
            return
        batch, count = self._a_batch, self._a_count
        self._a_batch, self._a_count = None, 0
        if self.a_factor is None:
            dt = self.factor_dtype or batch.dtype
            self.a_factor = self._new_identity(batch.shape[0], dt, batch.device)
        self._ema_(self.a_factor, batch, alpha, count)
        self._live['A'] = False  # the dense tensor changed in place

    def update_g_factor(self, alpha: float = 0.95) -> None:
        """Fold the accumulated batch factor into the running average."""
        if self._g_batch is None:
            return
        batch, count = self._g_batch, self._g_count
        self._g_batch, self._g_count = None, 0
        if self.g_factor is None:
            dt = self.factor_dtype or batch.dtype
            self.g_factor = self._new_identity(batch.shape[0], dt, batch.device)
        self._ema_(self.g_factor, batch, alpha, count)
        self._live['G'] = False  # the dense tensor changed in place

    # fused fast paths (one micro-batch per factor update)
    def save_and_update_a(self, input: list[torch.Tensor], alpha: float) -> None:
        self._save_and_update_a(input[0], alpha)

    def _save_and_update_a(self, a: torch.Tensor, alpha: float) -> None:
        if self._a_batch is not None or not (
            a.is_cuda and self._storage_dtype(a) == torch.float32
        ):
            self._save_a(a)
            self.update_a_factor(alpha)
            return
        if self._packed_update('A', a, 1.0 - alpha, alpha):
            return
        if self.a_factor is None:
            d = self.module.a_factor_shape[0]
            self.a_factor = self._new_identity(d, torch.float32, a.device)
        self.module.accumulate_a_factor(a, self.a_factor, 1.0 - alpha, alpha)

    def save_and_update_g(self, grad_output: tuple[torch.Tensor, ...], alpha: float) -> None:
        self._save_and_update_g(grad_output[0], alpha)

    def _save_and_update_g(self, g: torch.Tensor, alpha: float) -> None:
        if self._g_batch is not None or not (
            g.is_cuda and self._storage_dtype(g) == torch.float32
        ):
            self._save_g(g)
            self.update_g_factor(alpha)
            return
        unscale, dev_scale = self._g_unscale_parts(g.device)
        if self._packed_update('G', g, (1.0 - alpha) * unscale, alpha, dev_scale):
            return
        if self.g_factor is None:
            d = self.module.g_factor_shape[0]
            self.g_factor = self._new_identity(d, torch.float32, g.device)
        kw = {} if dev_scale is None else {'alpha_scale': dev_scale}
        self.module.accumulate_g_factor(
            g,
            self.g_factor,
            (1.0 - alpha) * unscale,
            alpha,
            **kw,
        )
