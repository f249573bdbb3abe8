"""Eigendecomposition K-FAC layer (reference ``kfac/layers/eigen.py:19-384``).

Preconditioning with the eigenbases QA, QG of the factors:

    V1 = QG^T [Wg | bg] QA
    V2 = V1 * dgda            (prediv: dgda = 1 / (dG (x) dA + damping))
       | V1 / (dG (x) dA + damping)
    P  = QG V2 QA^T

MI355X implementation: ``[Wg | bg] QA`` is formed as ``Wg QA[:-1] + bg (x)
QA[-1]`` (a GEMM on a row-slice of QA plus a rank-1 update) so the
concatenated gradient is never materialised; the four GEMMs run on hipBLASLt
into persistent fp32 buffers (``torch.mm(out=)``); the eigenvalue scaling is
a native in-place kernel.  Eigendecompositions are normally computed in
batches across layers by the preconditioner (``ops.linalg.eigh_many``) and
installed with ``set_a_eig`` / ``set_g_eig``; ``compute_a_inv`` /
``compute_g_inv`` remain for single-layer use.
"""
from __future__ import annotations

from typing import Any

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.layers.base import _nbytes
from distributed_kfac_pytorch_amd.layers.base import _resolve
from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.ops import linalg
from distributed_kfac_pytorch_amd.ops import precondition as pops
from distributed_kfac_pytorch_amd.parallel.comm import FutureType
from distributed_kfac_pytorch_amd.parallel.comm import get_rank


class KFACEigenLayer(KFACBaseLayer):
    """K-FAC layer preconditioning through factor eigendecompositions."""

    #: factors can go through the batched multi-layer eigensolver
    supports_batched_eigh = True

    def __init__(self, module: Any, *, prediv_eigenvalues: bool = False, **kwargs: Any) -> None:
        """Init KFACEigenLayer.

        Args:
            module (ModuleHelper): module helper.
            prediv_eigenvalues (bool): precompute ``1/(dG (x) dA + damping)``
                on the eigendecomposition worker (needs A and G colocated).
            **kwargs: ``KFACBaseLayer`` arguments.
        """
        super().__init__(module, **kwargs)
        self.prediv_eigenvalues = prediv_eigenvalues
        self._qa: torch.Tensor | FutureType | None = None
        self._qg: torch.Tensor | FutureType | None = None
        self._da: torch.Tensor | FutureType | None = None
        self._dg: torch.Tensor | FutureType | None = None
        self._dgda: torch.Tensor | FutureType | None = None
        self._tmp1: torch.Tensor | None = None
        self._tmp2: torch.Tensor | None = None
        # bf16 hi/lo planes of QA / QG for the grouped GEMMs (q_split)
        self._q_version = 0
        self._split_version = -1
        self._qa_hl: torch.Tensor | None = None
        self._qg_hl: torch.Tensor | None = None

    # ------------------------------------------------------------ properties
    @property
    def qa(self) -> torch.Tensor | None:
        self._qa = _resolve(self._qa)
        return self._qa

    @qa.setter
    def qa(self, v: torch.Tensor | FutureType | None) -> None:
        self._qa = v
        self._q_version += 1

    @property
    def qg(self) -> torch.Tensor | None:
        self._qg = _resolve(self._qg)
        return self._qg

    @qg.setter
    def qg(self, v: torch.Tensor | FutureType | None) -> None:
        self._qg = v
        self._q_version += 1

    @property
    def da(self) -> torch.Tensor | None:
        self._da = _resolve(self._da)
        return self._da

    @da.setter
    def da(self, v: torch.Tensor | FutureType | None) -> None:
        self._da = v

    @property
    def dg(self) -> torch.Tensor | None:
        self._dg = _resolve(self._dg)
        return self._dg

    @dg.setter
    def dg(self, v: torch.Tensor | FutureType | None) -> None:
        self._dg = v

    @property
    def dgda(self) -> torch.Tensor | None:
        self._dgda = _resolve(self._dgda)
        return self._dgda

    @dgda.setter
    def dgda(self, v: torch.Tensor | FutureType | None) -> None:
        self._dgda = v

    def memory_usage(self) -> dict[str, int]:
        sizes = super().memory_usage()
        sizes['a_inverses'] = _nbytes(self.qa) + _nbytes(self.da) + _nbytes(self._qa_hl)
        sizes['g_inverses'] = (
            _nbytes(self.qg) + _nbytes(self.dg) + _nbytes(self.dgda) + _nbytes(self._qg_hl)
        )
        return sizes

    @staticmethod
    def _split_into(buf: torch.Tensor | None, q: torch.Tensor) -> torch.Tensor:
        """q = hi + lo with hi = bf16_rn(q), lo = bf16_rn(q - hi) -- exactly
        the split csrc/gemm3.hip applies per tile -- into a persistent
        [rows, cols / 4, 8] bf16 buffer (hi x4, lo x4 per group of 4)."""
        r, c = q.shape
        shape = (r, c // 4, 8)
        if buf is None or tuple(buf.shape) != shape or buf.device != q.device:
            buf = torch.empty(shape, dtype=torch.bfloat16, device=q.device)
        qv = q.view(r, c // 4, 4)
        buf[:, :, :4].copy_(qv)
        buf[:, :, 4:].copy_(qv - buf[:, :, :4].float())
        return buf

    def q_split(self) -> tuple[torch.Tensor, torch.Tensor] | None:
        """Pre-split eigenbases for the grouped preconditioning GEMMs.

        The eigenbases change only at second-order updates (or when they
        are received by broadcast), so they are split into bf16 hi/lo
        planes once per update instead of in every GEMM tile of every step;
        the buffers keep their addresses (device tables, captured graphs).
        """
        qa, qg = self.qa, self.qg
        if qa is None or qg is None or qa.dtype != torch.float32 or qg.dtype != torch.float32:
            return None
        if not (qa.is_cuda and qa.is_contiguous() and qg.is_contiguous()):
            return None
        if qa.shape[1] % 4 or qg.shape[1] % 4:
            return None
        if self._split_version != self._q_version or self._qa_hl is None or self._qg_hl is None:
            if torch.cuda.is_current_stream_capturing():
                # never allocate / refresh inside a HIP-graph capture (the
                # buffers would live in the graph's private pool): the GEMMs
                # split in-kernel until the next eager refresh
                return None
            self._qa_hl = self._split_into(self._qa_hl, qa)
            self._qg_hl = self._split_into(self._qg_hl, qg)
            self._split_version = self._q_version
        return self._qa_hl, self._qg_hl

    # ------------------------------------------------------------ broadcasts
    def _bcast(self, t: torch.Tensor, src: int, group: dist.ProcessGroup | None,
               bucketed: bool) -> Any:
        if bucketed and self.tdc.bucket_cap_bytes > 0 and t.is_contiguous():
            # fused per-(group, src) broadcast; flushed by the preconditioner
            return self.tdc.broadcast_bucketed(t, src=src, group=group)
        return self.tdc.broadcast(t, src=src, group=group)

    def broadcast_a_inv(self, src: int, group: dist.ProcessGroup | None = None,
                        bucketed: bool = False) -> None:
        """Broadcast QA (and dA unless prediv) from the A inverse worker.
        ``bucketed`` fuses the tensors per (group, src) bucket; the caller
        must then call ``tdc.flush_broadcast_buckets()`` on every rank."""
        if self.qa is None or (not self.prediv_eigenvalues and self.da is None):
            if get_rank() == src:
                raise RuntimeError(
                    f'Attempt to broadcast A inv from src={src} but this rank '
                    'has not computed A inv yet.',
                )
            d = self.module.a_factor_shape[0]
            dev = self.module.device
            self.qa = torch.empty(d, d, device=dev, dtype=self.inv_dtype)
            self.da = torch.empty(d, device=dev, dtype=self.inv_dtype)
        self.qa = self._bcast(self.qa, src, group, bucketed)
        if not self.prediv_eigenvalues:
            assert self.da is not None
            self.da = self._bcast(self.da, src, group, bucketed)

    def broadcast_g_inv(self, src: int, group: dist.ProcessGroup | None = None,
                        bucketed: bool = False) -> None:
        """Broadcast QG and dG (or dGdA with prediv) from the G worker."""
        if (
            self.qg is None
            or (not self.prediv_eigenvalues and self.dg is None)
            or (self.prediv_eigenvalues and self.dgda is None)
        ):
            if get_rank() == src:
                raise RuntimeError(
                    f'Attempt to broadcast G inv from src={src} but this rank '
                    'has not computed G inv yet.',
                )
            g = self.module.g_factor_shape[0]
            a = self.module.a_factor_shape[0]
            dev = self.module.device
            self.qg = torch.empty(g, g, device=dev, dtype=self.inv_dtype)
            if not self.prediv_eigenvalues:
                self.dg = torch.empty(g, device=dev, dtype=self.inv_dtype)
            else:
                self.dgda = torch.empty(g, a, device=dev, dtype=self.inv_dtype)
        self.qg = self._bcast(self.qg, src, group, bucketed)
        if not self.prediv_eigenvalues:
            assert self.dg is not None
            self.dg = self._bcast(self.dg, src, group, bucketed)
        else:
            assert self.dgda is not None
            self.dgda = self._bcast(self.dgda, src, group, bucketed)

    # ---------------------------------------------------------- decomposition
    def _eig(self, factor: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        if self.symmetric_factors:
            return linalg.eigh(factor.to(torch.float32))
        d, q = torch.linalg.eig(factor.to(torch.float32))
        return d.real, q.real

    @staticmethod
    def _install(old: Any, new: torch.Tensor) -> torch.Tensor:
        """Copy ``new`` into the existing buffer when possible, so the
        second-order state keeps a fixed address across inverse updates
        (device tables and captured HIP graphs stay valid)."""
        if (
            isinstance(old, torch.Tensor)
            and old.shape == new.shape
            and old.dtype == new.dtype
            and old.device == new.device
            and old.is_contiguous()
        ):
            old.copy_(new)
            return old
        return new.contiguous()

    def set_a_eig(self, d: torch.Tensor, q: torch.Tensor) -> None:
        """Install an eigendecomposition of A (eigenvalues clamped at 0)."""
        self.qa = self._install(self.qa, q.to(self.inv_dtype))
        self._da_store = self._install(
            getattr(self, '_da_store', None),
            torch.clamp(d.to(self.inv_dtype), min=0.0),
        )
        self.da = self._da_store

    def set_g_eig(self, d: torch.Tensor, q: torch.Tensor, damping: float) -> None:
        """Install an eigendecomposition of G (and dGdA with prediv)."""
        self.qg = self._install(self.qg, q.to(self.inv_dtype))
        dg = torch.clamp(d.to(self.inv_dtype), min=0.0)
        if self.prediv_eigenvalues:
            assert self.da is not None
            dgda = torch.outer(dg, self.da).add_(damping).reciprocal_()
            self.dgda = self._install(self.dgda, dgda)
            self.dg = None
            self.da = None
        else:
            self._dg_store = self._install(getattr(self, '_dg_store', None), dg)
            self.dg = self._dg_store

    def compute_a_inv(self, damping: float = 0.001) -> None:
        """Eigendecompose A (rank must be the A inverse worker)."""
        if not isinstance(self.a_factor, torch.Tensor):
            raise RuntimeError('Cannot eigendecompose A before A has been computed')
        self.set_a_eig(*self._eig(self.a_factor))

    def compute_g_inv(self, damping: float = 0.001) -> None:
        """Eigendecompose G (and form dGdA if prediv)."""
        if not isinstance(self.g_factor, torch.Tensor):
            raise RuntimeError('Cannot eigendecompose G before G has been computed')
        if self.prediv_eigenvalues and self.da is None:
            raise RuntimeError('prediv_eigenvalues needs A eigenvalues first')
        self.set_g_eig(*self._eig(self.g_factor), damping=damping)

    # ----------------------------------------------------------- precondition
    def _buf(self, name: str, shape: tuple[int, int], dtype: torch.dtype, device: torch.device) -> torch.Tensor:
        t = getattr(self, name)
        if t is None or tuple(t.shape) != shape or t.dtype != dtype or t.device != device:
            t = torch.empty(shape, dtype=dtype, device=device)
            setattr(self, name, t)
        return t

    def preconditioned_grad(self, damping: float = 0.001) -> None:
        """Compute P = QG ((QG^T G QA) . S) QA^T into the grad buffer."""
        qa, qg = self.qa, self.qg
        if (
            qa is None
            or qg is None
            or (not self.prediv_eigenvalues and self.da is None)
            or (not self.prediv_eigenvalues and self.dg is None)
            or (self.prediv_eigenvalues and self.dgda is None)
        ):
            raise RuntimeError(
                'Eigendecompositions for both A and G have not been computed',
            )
        wg, bg, _ = self.precond_operands()
        dt = qa.dtype
        g_rows, a_cols = qg.shape[0], qa.shape[0]
        dev = qa.device
        t1 = self._buf('_tmp1', (g_rows, a_cols), dt, dev)
        t2 = self._buf('_tmp2', (g_rows, a_cols), dt, dev)
        # t1 = [Wg | bg] QA  (no concatenation)
        if bg is not None:
            torch.mm(wg.to(dt), qa[:-1], out=t1)
            t1.addr_(bg.reshape(-1).to(dt), qa[-1])
        else:
            torch.mm(wg.to(dt), qa, out=t1)
        torch.mm(qg.t(), t1, out=t2)  # V1
        if self.prediv_eigenvalues:
            pops.eigen_scale_(t2, dgda=self.dgda)
        else:
            pops.eigen_scale_(t2, dg=self.dg, da=self.da, damping=damping)
        torch.mm(qg, t2, out=t1)
        if dt == torch.float32:
            out = self.precond_out(dev)
            torch.mm(t1, qa.t(), out=out)
        else:
            out = (t1 @ qa.t()).to(torch.float32)
        self.grad = out
