"""K-FAC for ``nn.Embedding`` (new capability; the reference registers only
Linear / Conv2d).

An embedding lookup ``y = E[x]`` is a linear layer ``y = onehot(x) W^T`` with
``W = E^T`` (shape ``[dim, vocab]``).  Its input factor
``A = E[onehot onehot^T]`` is DIAGONAL -- the token frequencies -- so it is
stored as a length-``vocab`` vector (a dense 33k x 33k A would be 4.4 GB):

* accumulation: ``bincount`` of the token ids / N (no SYRK);
* eigendecomposition: ``QA = I``, ``dA = A`` (no solver call);
* inverse method: ``A_inv = 1 / (A + damping)``;
* preconditioning: ``P = QG ((QG^T grad) * 1/(dG (x) dA + damping))`` for
  eigen, ``P = G_inv grad diag(1/(A + damping))`` for inverse -- one GEMM
  fewer on each side than a dense layer, applied to ``W.grad = E.grad^T``.

G is the usual ``[dim, dim]`` covariance of the output gradient (SYRK).
Checkpoints store A as the 1-D frequency vector.  Enabled with
``KFACPreconditioner(..., register_embeddings=True)``; sparse embeddings and
``max_norm`` renormalisation are not supported.
"""
from __future__ import annotations

from typing import Any

import torch

from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.inverse import KFACInverseLayer
from distributed_kfac_pytorch_amd.layers.modules import ModuleHelper
from distributed_kfac_pytorch_amd.ops import factors as factor_ops


class EmbeddingModuleHelper(ModuleHelper):
    """Helper for ``torch.nn.Embedding`` with a diagonal A factor."""

    a_factor_is_diagonal = True

    def __init__(self, module: torch.nn.Embedding) -> None:
        if module.sparse:
            raise ValueError('sparse embeddings are not supported by K-FAC')
        super().__init__(module)

    @property
    def a_factor_shape(self) -> tuple[int, int]:
        v = self.module.num_embeddings
        return (v, v)

    @property
    def g_factor_shape(self) -> tuple[int, int]:
        d = self.module.embedding_dim
        return (d, d)

    def has_bias(self) -> bool:
        return False

    def accumulate_a_factor(self, a: torch.Tensor, out: torch.Tensor, alpha: float = 1.0, beta: float = 0.0) -> None:
        """``out = beta*out + alpha*counts/N`` (``out`` is a vector)."""
        ids = a.reshape(-1)
        n = max(ids.numel(), 1)
        counts = torch.bincount(ids, minlength=self.module.num_embeddings).to(out.dtype)
        if beta == 0.0:
            torch.mul(counts, alpha / n, out=out)
        else:
            out.mul_(beta).add_(counts, alpha=alpha / n)

    def accumulate_g_factor(self, g: torch.Tensor, out: torch.Tensor, alpha: float = 1.0,
                            beta: float = 0.0, alpha_scale: torch.Tensor | None = None) -> None:
        g2 = g.reshape(-1, g.shape[-1])
        n = max(g2.shape[0], 1)
        factor_ops.cov_accumulate_(out, g2, bias=False, alpha=alpha / n, beta=beta,
                                   alpha_scale=alpha_scale)

    def get_a_factor(self, a: torch.Tensor) -> torch.Tensor:
        out = torch.empty(self.module.num_embeddings, dtype=torch.float32, device=a.device)
        self.accumulate_a_factor(a, out, 1.0, 0.0)
        return out

    def weight_grad_matrix(self) -> torch.Tensor:
        """``W.grad = E.grad^T`` as [dim, vocab] (a view)."""
        return self.get_weight_grad().t()

    def _weight_from_matrix(self, wm: torch.Tensor) -> torch.Tensor:
        return wm.t()

    def write_grad(self, p: torch.Tensor, scale: torch.Tensor | float | None = None) -> None:
        g = self.module.weight.grad
        src = p if scale is None else p * scale
        if g is None:
            self.module.weight.grad = src.t().contiguous()
        else:
            g.copy_(src.t())


class _DiagonalAMixin:
    """Overrides for a vector-valued A factor (shared by eigen / inverse)."""

    supports_batched_eigh = False

    def _save_a(self, a: torch.Tensor) -> None:  # type: ignore[override]
        v = self.module.a_factor_shape[0]  # type: ignore[attr-defined]
        if self._a_batch is None:  # type: ignore[has-type]
            self._a_batch = torch.empty(v, dtype=torch.float32, device=a.device)
            self.module.accumulate_a_factor(a, self._a_batch, 1.0, 0.0)  # type: ignore[attr-defined]
            self._a_count = 1
        else:
            self.module.accumulate_a_factor(a, self._a_batch, 1.0, 1.0)  # type: ignore[attr-defined]
            self._a_count += 1

    def _save_and_update_a(self, a: torch.Tensor, alpha: float) -> None:  # type: ignore[override]
        self._save_a(a)
        self.update_a_factor(alpha)  # type: ignore[attr-defined]

    def update_a_factor(self, alpha: float = 0.95) -> None:  # type: ignore[override]
        if self._a_batch is None:
            return
        batch, count = self._a_batch, self._a_count
        self._a_batch, self._a_count = None, 0
        if self.a_factor is None:  # type: ignore[attr-defined]
            self.a_factor = torch.ones_like(batch)
        self.a_factor.mul_(alpha).add_(batch, alpha=(1.0 - alpha) / count)  # type: ignore[attr-defined]

    def reduce_a_factor(self, group: Any = None) -> None:  # type: ignore[override]
        if self.a_factor is None:  # type: ignore[attr-defined]
            raise RuntimeError('a_factor is None, cannot reduce')
        self.a_factor = self._allreduce()(  # type: ignore[attr-defined]
            self.a_factor, average=True, symmetric=False, group=group)

    def _a_to_ref(self, a: torch.Tensor) -> torch.Tensor:
        return a

    def _a_from_ref(self, a: torch.Tensor) -> torch.Tensor:
        return a.diagonal().contiguous() if a.dim() == 2 else a


class KFACEmbeddingEigenLayer(_DiagonalAMixin, KFACEigenLayer):
    """Eigen-method K-FAC for embeddings (QA = I)."""

    def compute_a_inv(self, damping: float = 0.001) -> None:
        if not isinstance(self.a_factor, torch.Tensor):
            raise RuntimeError('Cannot eigendecompose A before A has been computed')
        self.qa = None
        self._da_store = torch.clamp(self.a_factor.to(self.inv_dtype), min=0.0)
        self.da = self._da_store

    def broadcast_a_inv(self, src: int, group: Any = None, bucketed: bool = False) -> None:
        if self.da is None:
            v = self.module.a_factor_shape[0]
            self.da = torch.empty(v, device=self.module.device, dtype=self.inv_dtype)
        self.da = self.tdc.broadcast(self.da, src=src, group=group)

    def compute_g_inv(self, damping: float = 0.001) -> None:
        if not isinstance(self.g_factor, torch.Tensor):
            raise RuntimeError('Cannot eigendecompose G before G has been computed')
        if self.prediv_eigenvalues and self.da is None:
            raise RuntimeError('prediv_eigenvalues needs A eigenvalues first')
        d, q = self._eig(self.g_factor)
        self.set_g_eig(d, q, damping)

    def preconditioned_grad(self, damping: float = 0.001) -> None:
        qg = self.qg
        if qg is None or (self.prediv_eigenvalues and self.dgda is None) or (
            not self.prediv_eigenvalues and (self.da is None or self.dg is None)
        ):
            raise RuntimeError('Eigendecompositions for both A and G have not been computed')
        g = self.module.weight_grad_matrix().to(qg.dtype)
        v = qg.t() @ g
        if self.prediv_eigenvalues:
            v = v * self.dgda
        else:
            v = v / (torch.outer(self.dg, self.da) + damping)
        self.grad = (qg @ v).to(torch.float32)


class KFACEmbeddingInverseLayer(_DiagonalAMixin, KFACInverseLayer):
    """Inverse-method K-FAC for embeddings (A_inv diagonal)."""

    def compute_a_inv(self, damping: float = 0.001) -> None:
        if self.a_factor is None:
            raise RuntimeError('Cannot invert A before A has been computed')
        self.a_inv = (1.0 / (self.a_factor.to(torch.float32) + damping)).to(self.inv_dtype)

    def broadcast_a_inv(self, src: int, group: Any = None, bucketed: bool = False) -> None:
        if self.a_inv is None:
            v = self.module.a_factor_shape[0]
            self.a_inv = torch.empty(v, device=self.module.device, dtype=self.inv_dtype)
        self.a_inv = self.tdc.broadcast(self.a_inv, src=src, group=group)

    def preconditioned_grad(self, damping: float = 0.001) -> None:
        if self.a_inv is None or self.g_inv is None:
            raise RuntimeError('Cannot precondition gradient before A and G have been inverted')
        g = self.module.weight_grad_matrix().to(self.g_inv.dtype)
        self.grad = ((self.g_inv @ g) * self.a_inv[None, :]).to(torch.float32)
