"""Module adapters: per-module factor math and gradient views.

Reference: ``kfac/layers/modules.py:13-237`` (``ModuleHelper``,
``LinearModuleHelper``, ``Conv2dModuleHelper``).  The reference API
(``get_a_factor`` / ``get_g_factor`` returning a fresh covariance,
``get_grad`` / ``set_grad`` with the bias as an extra column) is kept.  The
MI355X hot path uses the in-place forms instead:

* ``accumulate_a_factor(a, out, alpha, beta)`` /
  ``accumulate_g_factor(g, out, alpha, beta)``: ``out = beta*out + alpha*
  scale*Xt^T Xt`` in one SYRK launch, no bias-column cat, no clone of the
  activation, no im2col for 1x1 convs in channels_last.
* ``weight_grad_matrix()`` / ``write_grad(P, scale)``: zero-copy views of the
  parameter gradients in the factor's column order and an in-place scaled
  write back (no cat / split / contiguous).

Conv2d column order.  With a channels_last (NHWC) input, factors are kept in
the "natural" (kh, kw, c) column order, which is the physical layout of a
channels_last weight gradient ``[out][kh][kw][c]`` -- so both the patch
extraction and the gradient view are straight copies/views.  Otherwise the
reference (c, kh, kw) order is used.  ``state_dict`` always emits the
reference order (see ``KFACBaseLayer.state_dict``), so checkpoints are
interchangeable with the reference.
"""
from __future__ import annotations

import torch

from distributed_kfac_pytorch_amd.layers.utils import append_bias_ones
from distributed_kfac_pytorch_amd.layers.utils import get_cov
from distributed_kfac_pytorch_amd.ops import factors as factor_ops


class ModuleHelper:
    """Interface between a ``torch.nn.Module`` and a K-FAC layer."""

    def __init__(self, module: torch.nn.Module):
        self.module = module

    def __repr__(self) -> str:
        return f'{self.__class__.__name__}({self.module!r})'

    @property
    def a_factor_shape(self) -> tuple[int, int]:
        raise NotImplementedError

    @property
    def g_factor_shape(self) -> tuple[int, int]:
        raise NotImplementedError

    @property
    def device(self) -> torch.device:
        return next(self.module.parameters()).device

    # ---------------------------------------------------------------- factors
    def accumulate_a_factor(
        self,
        a: torch.Tensor,
        out: torch.Tensor,
        alpha: float = 1.0,
        beta: float = 0.0,
    ) -> None:
        raise NotImplementedError

    def accumulate_g_factor(
        self,
        g: torch.Tensor,
        out: torch.Tensor,
        alpha: float = 1.0,
        beta: float = 0.0,
        alpha_scale: torch.Tensor | None = None,
    ) -> None:
        raise NotImplementedError

    def get_a_factor(self, a: torch.Tensor) -> torch.Tensor:
        """Batch A factor of one forward input (fresh tensor)."""
        d = self.a_factor_shape[0]
        out = torch.empty(d, d, dtype=_acc_dtype(a), device=a.device)
        self.accumulate_a_factor(a, out, 1.0, 0.0)
        return out

    def get_g_factor(self, g: torch.Tensor) -> torch.Tensor:
        """Batch G factor of one output gradient (fresh tensor)."""
        d = self.g_factor_shape[0]
        out = torch.empty(d, d, dtype=_acc_dtype(g), device=g.device)
        self.accumulate_g_factor(g, out, 1.0, 0.0)
        return out

    # ------------------------------------------------------------------ grads
    def has_bias(self) -> bool:
        return getattr(self.module, 'bias', None) is not None

    def has_symmetric_factors(self) -> bool:
        return True

    def get_weight_grad(self) -> torch.Tensor:
        g = self.module.weight.grad
        if g is None:
            raise RuntimeError(
                f'{self.module!r} has no weight gradient; run backward first',
            )
        return g

    def get_bias_grad(self) -> torch.Tensor:
        g = self.module.bias.grad
        if g is None:
            raise RuntimeError(
                f'{self.module!r} has no bias gradient; run backward first',
            )
        return g

    def weight_grad_matrix(self) -> torch.Tensor:
        """Weight gradient as [out, cols] in the factor column order."""
        w = self.get_weight_grad()
        return w.reshape(w.shape[0], -1)

    def get_grad(self) -> torch.Tensor:
        """``[W_grad | b_grad]`` as one [out, cols(+1)] matrix (a copy when
        there is a bias)."""
        g = self.weight_grad_matrix()
        if self.has_bias():
            g = torch.cat([g, self.get_bias_grad().reshape(-1, 1)], dim=1)
        return g

    def _weight_from_matrix(self, wm: torch.Tensor) -> torch.Tensor:
        return wm.reshape(self.module.weight.shape)

    def set_grad(self, grad: torch.Tensor) -> None:
        """Replace the module gradients with ``grad`` ([out, cols(+1)])."""
        if self.has_bias():
            wm = grad[:, :-1]
            self.module.bias.grad = grad[:, -1].reshape(
                self.module.bias.shape,
            ).contiguous()
        else:
            wm = grad
        self.module.weight.grad = self._weight_from_matrix(
            wm.contiguous(),
        ).contiguous(memory_format=_memory_format(self.module.weight))

    def write_grad(
        self,
        p: torch.Tensor,
        scale: torch.Tensor | float | None = None,
    ) -> None:
        """In place: weight/bias grads = scale * P (P in factor order)."""
        from distributed_kfac_pytorch_amd.ops import precondition as pops

        wg = self.module.weight.grad
        if wg is None:
            self.set_grad(p if scale is None else p * scale)
            return
        wm = self.weight_grad_matrix()
        bg = self.get_bias_grad() if self.has_bias() else None
        aliased = wm.data_ptr() == wg.data_ptr() and wm.is_contiguous()
        pops.apply_grad_(p, wm, bg, scale)
        if not aliased:  # the view had to copy: write it back
            wg.copy_(self._weight_from_matrix(wm))


def _acc_dtype(x: torch.Tensor) -> torch.dtype:
    """Accumulation dtype for a factor computed from ``x``: fp32 for half
    types (the MFMA accumulator precision), the input dtype otherwise."""
    if x.dtype in (torch.float16, torch.bfloat16):
        return torch.float32
    return x.dtype


def _memory_format(t: torch.Tensor) -> torch.memory_format:
    if t.dim() == 4 and factor_ops.is_channels_last(t) and not t.is_contiguous():
        return torch.channels_last
    return torch.contiguous_format


class LinearModuleHelper(ModuleHelper):
    """Helper for ``torch.nn.Linear`` (and subclasses)."""

    @property
    def a_factor_shape(self) -> tuple[int, int]:
        x = self.module.weight.shape[1] + int(self.has_bias())
        return (x, x)

    @property
    def g_factor_shape(self) -> tuple[int, int]:
        x = self.module.weight.shape[0]
        return (x, x)

    def accumulate_a_factor(
        self,
        a: torch.Tensor,
        out: torch.Tensor,
        alpha: float = 1.0,
        beta: float = 0.0,
    ) -> None:
        a2 = a.reshape(-1, a.shape[-1])
        n = max(a2.shape[0], 1)
        factor_ops.cov_accumulate_(
            out,
            a2,
            bias=self.has_bias(),
            alpha=alpha / n,
            beta=beta,
        )

    def accumulate_g_factor(
        self,
        g: torch.Tensor,
        out: torch.Tensor,
        alpha: float = 1.0,
        beta: float = 0.0,
        alpha_scale: torch.Tensor | None = None,
    ) -> None:
        g2 = g.reshape(-1, g.shape[-1])
        n = max(g2.shape[0], 1)
        factor_ops.cov_accumulate_(out, g2, bias=False, alpha=alpha / n, beta=beta,
                                   alpha_scale=alpha_scale)

    def get_a_factor(self, a: torch.Tensor) -> torch.Tensor:
        if a.is_cuda:
            return super().get_a_factor(a)
        # exact reference arithmetic on CPU (kfac/layers/modules.py:123-132)
        a = a.reshape(-1, a.shape[-1])
        if self.has_bias():
            a = append_bias_ones(a)
        return get_cov(a)

    def get_g_factor(self, g: torch.Tensor) -> torch.Tensor:
        if g.is_cuda:
            return super().get_g_factor(g)
        return get_cov(g.reshape(-1, g.shape[-1]))


class Conv2dModuleHelper(ModuleHelper):
    """Helper for ``torch.nn.Conv2d`` (zero padding, any stride; dilation
    and groups must be 1 -- such convs are not registered)."""

    def __init__(self, module: torch.nn.Conv2d):
        super().__init__(module)
        if tuple(module.dilation) != (1, 1) or module.groups != 1:
            raise ValueError(
                'K-FAC Conv2d factors require dilation=1 and groups=1',
            )
        if getattr(module, 'padding_mode', 'zeros') != 'zeros':
            raise ValueError('K-FAC Conv2d factors require zero padding')
        self._natural: bool | None = None

    @property
    def kernel(self) -> tuple[int, int]:
        k = self.module.kernel_size
        return (int(k[0]), int(k[1]))

    @property
    def stride(self) -> tuple[int, int]:
        s = self.module.stride
        return (int(s[0]), int(s[1]))

    @property
    def padding(self) -> tuple[int, int]:
        p = self.module.padding
        if isinstance(p, str):
            if p == 'valid':
                return (0, 0)
            raise ValueError("padding='same' is not supported by K-FAC")
        return (int(p[0]), int(p[1]))

    @property
    def natural_order(self) -> bool:
        """True when factors use the (kh, kw, c) column order.

        Decided once, on first use, from the memory format of the weight:
        a channels_last conv (``model.to(memory_format=torch.channels_last)``)
        gets natural order, anything else the reference order.  1x1 kernels
        have identical orders.
        """
        if self._natural is None:
            w = self.module.weight
            self._natural = bool(
                self.kernel != (1, 1)
                and factor_ops.is_channels_last(w)
                and not w.is_contiguous(),
            )
        return self._natural

    @property
    def a_factor_shape(self) -> tuple[int, int]:
        kh, kw = self.kernel
        x = self.module.in_channels * kh * kw + int(self.has_bias())
        return (x, x)

    @property
    def g_factor_shape(self) -> tuple[int, int]:
        x = self.module.out_channels
        return (x, x)

    def _prepare_input(self, a: torch.Tensor) -> torch.Tensor:
        if self.natural_order and not factor_ops.is_channels_last(a):
            a = a.contiguous(memory_format=torch.channels_last)
        return a

    def _dense_view(self, a: torch.Tensor) -> bool:
        """1x1 / stride 1 / no padding on NHWC: the patch matrix is a free
        view of the input (plain SYRK, see factor_ops.conv_patches)."""
        return (
            self.kernel == (1, 1)
            and self.stride == (1, 1)
            and self.padding == (0, 0)
            and factor_ops.is_channels_last(a)
        )

    def accumulate_a_factor(
        self,
        a: torch.Tensor,
        out: torch.Tensor,
        alpha: float = 1.0,
        beta: float = 0.0,
    ) -> None:
        a = self._prepare_input(a)
        if (
            self.natural_order or self.kernel == (1, 1)
        ) and not self._dense_view(a):
            oh, ow = factor_ops.conv_out_hw(a.shape[2], a.shape[3], self.kernel,
                                            self.stride, self.padding)
            n = max(a.shape[0] * oh * ow, 1)
            if factor_ops.conv_cov_accumulate_(
                out, a, self.kernel, self.stride, self.padding,
                bias=self.has_bias(),
                alpha=alpha / (n * float(oh * ow) ** 2),
                beta=beta,
            ):
                return
        patches, spatial = factor_ops.conv_patches(
            a,
            self.kernel,
            self.stride,
            self.padding,
            natural=self.natural_order,
        )
        n = max(patches.shape[0], 1)
        factor_ops.cov_accumulate_(
            out,
            patches,
            bias=self.has_bias(),
            alpha=alpha / (n * float(spatial) ** 2),
            beta=beta,
        )

    def accumulate_g_factor(
        self,
        g: torch.Tensor,
        out: torch.Tensor,
        alpha: float = 1.0,
        beta: float = 0.0,
        alpha_scale: torch.Tensor | None = None,
    ) -> None:
        spatial = g.shape[2] * g.shape[3]
        rows = factor_ops.rows_nhwc(g)
        n = max(rows.shape[0], 1)
        factor_ops.cov_accumulate_(
            out,
            rows,
            bias=False,
            alpha=alpha / (n * float(spatial) ** 2),
            beta=beta,
            alpha_scale=alpha_scale,
        )

    def get_a_factor(self, a: torch.Tensor) -> torch.Tensor:
        if a.is_cuda:
            return super().get_a_factor(a)
        # reference arithmetic on CPU (kfac/layers/modules.py:170-178)
        a = self._prepare_input(a)
        patches, spatial = factor_ops.conv_patches(
            a,
            self.kernel,
            self.stride,
            self.padding,
            natural=self.natural_order,
        )
        if self.has_bias():
            patches = append_bias_ones(patches)
        return get_cov(patches / spatial)

    def get_g_factor(self, g: torch.Tensor) -> torch.Tensor:
        if g.is_cuda:
            return super().get_g_factor(g)
        spatial = g.shape[2] * g.shape[3]
        rows = factor_ops.rows_nhwc(g)
        return get_cov(rows / spatial)

    def weight_grad_matrix(self) -> torch.Tensor:
        w = self.get_weight_grad()
        if self.natural_order:
            return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
        return w.reshape(w.shape[0], -1)

    def _weight_from_matrix(self, wm: torch.Tensor) -> torch.Tensor:
        o, c, kh, kw = self.module.weight.shape
        if self.natural_order:
            return wm.reshape(o, kh, kw, c).permute(0, 3, 1, 2)
        return wm.reshape(o, c, kh, kw)

    # --------------------------------------------------- checkpoint ordering
    def a_to_reference_order(self, a: torch.Tensor) -> torch.Tensor:
        """Permute a natural-order A factor to the reference (c, kh, kw)."""
        if not self.natural_order:
            return a
        perm = self._perm(a.device)
        return a.index_select(0, perm).index_select(1, perm)

    def a_from_reference_order(self, a: torch.Tensor) -> torch.Tensor:
        if not self.natural_order:
            return a
        inv = torch.argsort(self._perm(a.device))
        return a.index_select(0, inv).index_select(1, inv)

    def _perm(self, device: torch.device) -> torch.Tensor:
        # reference column r = c*KK + k  <-  natural column k*C + c
        kh, kw = self.kernel
        c = self.module.in_channels
        kk = kh * kw
        r = torch.arange(c * kk, device=device)
        nat = (r % kk) * c + r // kk
        if self.has_bias():
            nat = torch.cat([nat, torch.tensor([c * kk], device=device)])
        return nat
