"""Gradient preconditioning (K-HIP-4) and the device-side KL clip (K-HIP-7).

The GEMM chain ``QG^T [Wg | bg] QA -> scale -> QG (.) QA^T`` of every layer
runs as four grouped bf16x3 MFMA launches (``GroupedPrecondition``,
csrc/gemm3.hip) on CUDA; the per-layer ``torch.mm(..., out=)`` chain is the
fallback (CPU, ``KFAC_PRECOND_GEMM=torch``, unsupported layer types).
Everything between and after the GEMMs is a native kernel here, so a K-FAC
step performs no host synchronisation:

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
from typing import Any
from typing import Callable

import torch

from distributed_kfac_pytorch_amd.ops._native import native
from distributed_kfac_pytorch_amd.ops._native import use_native
from distributed_kfac_pytorch_amd.utils.env import getenv


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


def _used_here(tab: torch.Tensor) -> torch.Tensor:
    """Mark an eagerly uploaded descriptor table as used by the current
    stream before a launch reads it, so the caching allocator does not hand
    its block to another stream's allocation while that launch is queued
    (a table may be uploaded on one stream and launched on another, e.g. the
    precondition GEMMs issued from the early side stream).  Tables built
    during a capture live in persistent device slots and need no marking."""
    if tab.is_cuda and not torch.cuda.is_current_stream_capturing():
        tab.record_stream(torch.cuda.current_stream(tab.device))
    return tab


class _TableCache:
    """Small LRU of device descriptor tables keyed by operand addresses,
    with the pinned host staging buffers they are uploaded from.

    A table built inside a HIP-graph capture (``graphs.GraphedTrainStep``:
    the captured backward produces gradients at new addresses) is written to
    the persistent device twin of its staging slot -- allocated eagerly,
    outside every graph pool -- and uploaded once, eagerly, right after the
    capture (``_native.flush_table_uploads``); no copy node is captured.
    Pinned and device slots cannot be allocated while a capture is running,
    so they are allocated the first time they are needed outside a capture
    and recycled after that.

    Staging reuse is fenced: an eager upload records a HIP event on the
    stream that runs its H2D copy, and a buffer whose entry is evicted is
    parked until that event has completed -- the host never rewrites a
    staging buffer a queued copy has yet to read (the host runs ahead of the
    GPU by whole steps).  Entries referenced by a captured graph are never
    evicted: those built or looked up during a capture (sticky), and those a
    caller pins explicitly (``pin`` / ``unpin``, used by ``StepGraphs``
    whose tables are built just before its capture).
    """

    SLOT_BYTES = 1 << 16  # >= 500 layers of descriptors per table

    def __init__(self, size: int = 8, slots_per_entry: int = 1) -> None:
        self.size = size
        self.per = slots_per_entry
        # key -> (value, slots, event | None)
        self._d: dict = {}
        # clean staging buffers (no pending H2D copy reads them)
        self._free: list[torch.Tensor] = []
        # evicted buffers whose last copy may still be queued: (buf, event)
        self._parked: list[tuple[torch.Tensor, Any]] = []
        self._sticky: set = set()
        self._pins: dict = {}
        # device twins of the staging slots (kept alive here)
        self._dev_slots: list[torch.Tensor] = []
        self._slot_hosts: list[torch.Tensor] = []

    def __del__(self) -> None:
        # drop the native slot registry's references to this cache's twins
        try:
            lib = native()
            if lib is not None and hasattr(lib, 'unregister_table_slot'):
                for h in self._slot_hosts:
                    lib.unregister_table_slot(h)
        except Exception:  # noqa: BLE001  (interpreter shutdown)
            pass

    @staticmethod
    def _capturing() -> bool:
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()

    def _held(self, key: tuple) -> bool:
        return key in self._sticky or self._pins.get(key, 0) > 0

    def pin(self, key: tuple | None) -> None:
        if key is not None and key in self._d:
            self._pins[key] = self._pins.get(key, 0) + 1

    def unpin(self, key: tuple | None) -> None:
        if key is None:
            return
        n = self._pins.get(key, 0) - 1
        if n > 0:
            self._pins[key] = n
        else:
            self._pins.pop(key, None)

    def get(self, key: tuple) -> Any:
        v = self._d.pop(key, None)
        if v is not None:
            self._d[key] = v
            if self._capturing():
                self._sticky.add(key)
            return v[0]
        return None

    def _unpark(self, wait: bool) -> None:
        keep = []
        for buf, ev in self._parked:
            if ev is None or ev.query():
                self._free.append(buf)
            elif wait:
                ev.synchronize()
                self._free.append(buf)
            else:
                keep.append((buf, ev))
        self._parked = keep

    def reserve(self) -> list[torch.Tensor | None]:
        """Staging buffers for one new entry (None: let the builder
        allocate, which is only possible outside a capture)."""
        while len(self._d) - sum(1 for k in self._d if self._held(k)) >= self.size:
            victim = next((k for k in self._d if not self._held(k)), None)
            if victim is None:
                break
            _, slots, ev = self._d.pop(victim)
            self._parked += [(t, ev) for t in slots if t is not None]
        capturing = self._capturing()
        if not capturing and torch.cuda.is_available():
            # a parked buffer is reused only once its last copy has run
            self._unpark(wait=len(self._free) < self.per)
            # top up so that a later capture never has to allocate: each
            # pinned staging slot gets a persistent device twin (outside any
            # graph pool) that a table built during a capture is written to
            # (csrc/bindings.cpp upload_table / register_table_slot)
            while len(self._free) < self.per * self.size:
                host = torch.empty(self.SLOT_BYTES, dtype=torch.uint8, pin_memory=True)
                lib = native()
                if lib is not None and hasattr(lib, 'register_table_slot'):
                    dev = torch.empty(self.SLOT_BYTES, dtype=torch.uint8,
                                      device=torch.device('cuda', torch.cuda.current_device()))
                    lib.register_table_slot(host, dev)
                    self._dev_slots.append(dev)
                    self._slot_hosts.append(host)
                self._free.append(host)
        out: list[torch.Tensor | None] = []
        for _ in range(self.per):
            out.append(self._free.pop() if self._free else None)
        return out

    def put(self, key: tuple, value: Any, slots: list) -> Any:
        ev = None
        if self._capturing():
            self._sticky.add(key)
        elif torch.cuda.is_available() and any(t is not None for t in slots):
            # the uploads were enqueued on the current stream
            ev = torch.cuda.Event()
            ev.record()
        self._d[key] = (value, slots, ev)
        return value


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
        self._tables = _TableCache(slots_per_entry=1)
        self._acc: torch.Tensor | None = None
        self._retired: list[torch.Tensor] = []
        self._scale: torch.Tensor | None = None
        self._params: torch.Tensor | None = None
        self._param_vals: tuple[float, float] | None = None
        self._sum: torch.Tensor | None = None
        self._n = 0

    def _buffers(self, device: torch.device, nparts: int) -> None:
        if self._acc is None or self._acc.device != device:
            self._acc = None
            self._scale = torch.ones(1, dtype=torch.float32, device=device)
            self._params = torch.zeros(2, dtype=torch.float32, device=device)
            self._param_vals = None
        if self._acc is None or self._acc.numel() < nparts:
            # one fp64 KL partial per block (summed in a fixed order).  A
            # replaced buffer is kept alive: a captured graph may still read it
            if self._acc is not None:
                self._retired.append(self._acc)
            self._acc = torch.zeros(max(nparts, 256), dtype=torch.float64, device=device)

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
        ps, ws, bs, bsc = [], [], [], []
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
            # weight of the bias in the KL sum (1/mp for a bias replicated
            # over a tensor-parallel group, see neox/layer.py)
            bsc.append(float(getattr(layer, 'kl_bias_scale', 1.0)))
            key.append((
                p.data_ptr(), tuple(p.shape), p.stride(0), wm.data_ptr(),
                tuple(wm.shape), wm.dtype, None if bg is None else bg.data_ptr(),
                None if bg is None else bg.dtype, bsc[-1],
            ))
        key_t = tuple(key)
        if key_t != self._key:
            entry = self._tables.get(key_t)
            if entry is None:
                slots = self._tables.reserve()
                entry = self._tables.put(
                    key_t, lib.build_layer_table(ps, ws, bs, slots[0], bsc), slots)
            self._table, self._blocks, _ = entry
            self._key = key_t
        self._n = len(ps)
        self._buffers(ps[0].device, self._blocks)
        if kl_clip is not None:
            vals = (float(kl_clip), float(lr))
            if vals != self._param_vals:
                self._params[0].fill_(vals[0])
                self._params[1].fill_(vals[1])
                self._param_vals = vals
        return True

    def hold(self) -> tuple | None:
        """Pin the current table (a graph about to be captured uses it);
        returns the handle for ``release``."""
        self._tables.pin(self._key)
        return self._key

    def release(self, key: tuple | None) -> None:
        self._tables.unpin(key)

    def launch(self, with_kl: bool, reduce_fn: Callable[[torch.Tensor], None] | None = None) -> None:
        """The three (or one, without KL clip) multi-tensor launches.

        ``reduce_fn`` (tensor parallelism): the per-block partials are first
        folded into one fp64 per-rank sum, ``reduce_fn`` all-reduces that
        1-element tensor in place over the model-parallel group, and the
        scale is finalised from the global sum -- one scalar collective for
        the whole model."""
        lib = native()
        _used_here(self._table)
        if not with_kl:
            lib.apply_multi(self._table, self._n, self._blocks, None)
            return
        lib.kl_dot_multi(self._table, self._n, self._blocks, self._acc)
        if reduce_fn is None:
            lib.kl_finalize_dev(self._acc, self._blocks, self._params, self._scale)
        else:
            if self._sum is None or self._sum.device != self._acc.device:
                self._sum = torch.zeros(1, dtype=torch.float64, device=self._acc.device)
            lib.kl_reduce_partials(self._acc, self._blocks, self._sum)
            reduce_fn(self._sum)
            lib.kl_finalize_dev(self._sum, 1, self._params, self._scale)
        lib.apply_multi(self._table, self._n, self._blocks, self._scale)

    def run(
        self,
        layers: list,
        kl_clip: float | None,
        lr: float,
        reduce_fn: Callable[[torch.Tensor], None] | None = None,
    ) -> bool:
        """prepare + launch for an eagerly preconditioned step."""
        if not self.prepare(layers, kl_clip, lr):
            return False
        self.launch(kl_clip is not None, reduce_fn)
        for layer in layers:
            layer.grad = None
        return True


def presplit_enabled() -> bool:
    return getenv('KFAC_GEMM3_PRESPLIT', '0') == '1'


def grouped_gemm_enabled() -> bool:
    """``KFAC_PRECOND_GEMM=torch`` keeps the per-layer hipBLASLt fp32 chain;
    otherwise a grouped bf16x3 MFMA kernel runs (``grouped_gemm_mode``)."""
    return getenv('KFAC_PRECOND_GEMM', 'bf16x3').lower() != 'torch'


class GroupedPrecondition:
    """All layers' preconditioning GEMM chains in four grouped launches.

    Eigen layers (reference ``kfac/layers/eigen.py:349-384``)::

        T1: t1 = [Wg | bg] QA          (bias column read from bg in place)
        T2: t2 = (QG^T t1) (.) S       (S = dGdA, or 1/(dG (x) dA + damping))
        T3: t1 = QG t2
        T4: P  = t1 QA^T               (P = the layer's persistent grad buffer)

    Inverse layers (``kfac/layers/inverse.py:214-233``) use T1 with
    ``A^-1`` and write ``P = G^-1 t1`` in T3.  Each launch covers every
    layer (csrc/gemm3.hip), so a ResNet-50 step issues 4 GEMM launches
    instead of ~220.  Tables are cached on the operand addresses (all
    persistent between second-order updates).
    """

    def __init__(self) -> None:
        self._key: tuple | None = None
        self._tables: list = []
        self._cache = _TableCache(slots_per_entry=4)

    @staticmethod
    def _operands(layer: Any) -> tuple | None:
        from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
        from distributed_kfac_pytorch_amd.layers.inverse import KFACInverseLayer

        # only the stock layer math: subclasses that override the
        # preconditioning (embedding) keep their path; tensor-parallel NeoX
        # layers run the stock math on their gathered operands
        # (``stock_precondition_math``)
        if type(layer).preconditioned_grad not in (
            KFACEigenLayer.preconditioned_grad, KFACInverseLayer.preconditioned_grad,
        ) and not getattr(layer, 'stock_precondition_math', False):
            return None
        wm, bg, stable = layer.precond_operands()
        if wm is None or not stable or not wm.is_cuda or wm.dtype != torch.float32:
            return None
        if bg is not None and (bg.dtype != torch.float32 or not bg.is_contiguous()):
            return None
        if isinstance(layer, KFACEigenLayer):
            qa, qg = layer.qa, layer.qg
            if qa is None or qg is None or qa.dtype != torch.float32 or qg.dtype != torch.float32:
                return None
            if layer.prediv_eigenvalues:
                if layer.dgda is None or layer.dgda.dtype != torch.float32:
                    return None
            elif layer.dg is None or layer.da is None:
                return None
            return ('eigen', wm, bg, qa, qg)
        if isinstance(layer, KFACInverseLayer):
            a_inv, g_inv = layer.a_inv, layer.g_inv
            if a_inv is None or g_inv is None or a_inv.dtype != torch.float32 \
                    or g_inv.dtype != torch.float32:
                return None
            # (F + damping I)^-1 is symmetric: a column-major result (e.g.
            # from cholesky_inverse) is used through its transpose
            a_inv = a_inv if a_inv.stride(1) == 1 else a_inv.t()
            g_inv = g_inv if g_inv.stride(1) == 1 else g_inv.t()
            if a_inv.stride(1) != 1 or g_inv.stride(1) != 1:
                return None
            return ('inverse', wm, bg, a_inv, g_inv)
        return None

    @staticmethod
    def _splits(layer: Any) -> tuple | None:
        """bf16 hi/lo planes of the layer's constant operands (eigenbases),
        refreshed once per second-order update, or None.

        Opt-in (``KFAC_GEMM3_PRESPLIT=1``): on MI355X the in-kernel split
        measured the same within run-to-run noise (ResNet-50 plain graph step
        8.88 / 9.11 ms pre-split vs 9.08 / 9.10 ms in-kernel, same box) --
        the grouped GEMM is bound by its operand loads and LDS traffic, not
        by the split -- and the planes cost as much memory as the bases."""
        if not presplit_enabled():
            return None
        fn = getattr(layer, 'q_split', None)
        return fn() if fn is not None else None

    def prepare(self, layers: list, damping: float) -> bool:
        lib = native()
        if lib is None or not layers or not grouped_gemm_enabled():
            return False
        ops = []
        for layer in layers:
            o = self._operands(layer)
            if o is None:
                return False
            ops.append(o)
        t = [[] for _ in range(4)]  # per table: list of operand tuples
        key = [damping]
        outs: list[torch.Tensor] = []
        for layer, (kind, wm, bg, fa, fg) in zip(layers, ops):
            g, a = fg.shape[0], fa.shape[0]
            dev = fa.device
            hl = self._splits(layer) if kind == 'eigen' else None
            qa_hl, qg_hl = hl if hl is not None else (None, None)
            t1 = layer._buf('_tmp1', (g, a), torch.float32, dev) if kind == 'eigen' \
                else self._inv_tmp(layer, (g, a), dev)
            out = layer.precond_out(dev)
            if tuple(out.shape) != (g, a):
                return False
            outs.append(out)
            key.append((kind, wm.data_ptr(), None if bg is None else bg.data_ptr(),
                        fa.data_ptr(), fg.data_ptr(), t1.data_ptr(), out.data_ptr(), g, a,
                        None if qa_hl is None else (qa_hl.data_ptr(), qg_hl.data_ptr())))
            # T1: [Wg | bg] @ QA  (or A^-1); rows: (A, A_extra, B, C, S, dg, da,
            # damping, A_hl, B_hl)
            t[0].append((wm, bg, fa, t1, None, None, None, 0.0, None, qa_hl))
            if kind == 'eigen':
                t2 = layer._buf('_tmp2', (g, a), torch.float32, dev)
                key.append((t2.data_ptr(), layer.prediv_eigenvalues,
                            None if layer.dgda is None else layer.dgda.data_ptr(),
                            None if layer.dg is None else layer.dg.data_ptr(),
                            None if layer.da is None else layer.da.data_ptr()))
                if layer.prediv_eigenvalues:
                    t[1].append((fg, None, t1, t2, layer.dgda, None, None, 0.0, qg_hl, None))
                else:
                    t[1].append((fg, None, t1, t2, None, layer.dg, layer.da, float(damping),
                                 qg_hl, None))
                t[2].append((fg, None, t2, t1, None, None, None, 0.0, qg_hl, None))
                t[3].append((t1, None, fa, out, None, None, None, 0.0, None, qa_hl))
            else:
                t[2].append((fg, None, t1, out, None, None, None, 0.0, None, None))
        key_t = tuple(key)
        if key_t != self._key:
            tables = self._cache.get(key_t)
            if tables is None:
                flags = [(True, False), (False, False), (True, False), (True, True)]
                slots = self._cache.reserve()
                tables = []
                for rows, (akc, bkc), slot in zip(t, flags, slots):
                    if not rows:
                        tables.append(None)
                        continue
                    cols = list(zip(*rows))
                    tab, tiles, host = lib.build_gemm_table(
                        list(cols[0]), list(cols[1]), list(cols[2]), list(cols[3]),
                        list(cols[4]), list(cols[5]), list(cols[6]), list(cols[7]), akc, bkc,
                        slot, list(cols[8]), list(cols[9]),
                    )
                    tables.append((tab, len(rows), tiles, akc, bkc, host))
                self._cache.put(key_t, tables, slots)
            self._tables = tables
            self._key = key_t
        self._layers = layers
        self._outs = outs
        return True

    @staticmethod
    def _inv_tmp(layer: Any, shape: tuple[int, int], dev: torch.device) -> torch.Tensor:
        t = getattr(layer, '_gtmp', None)
        if t is None or tuple(t.shape) != shape or t.device != dev:
            t = torch.empty(shape, dtype=torch.float32, device=dev)
            layer._gtmp = t
        return t

    def hold(self) -> tuple | None:
        """Pin the current tables (a graph about to be captured uses
        them); returns the handle for ``release``."""
        self._cache.pin(self._key)
        return self._key

    def release(self, key: tuple | None) -> None:
        self._cache.unpin(key)

    def launch(self) -> None:
        lib = native()
        for entry in self._tables:
            if entry is not None:
                tab, n, tiles, akc, bkc, _ = entry
                lib.gemm3_grouped(_used_here(tab), n, tiles, akc, bkc)

    def run(self, layers: list, damping: float) -> bool:
        """prepare + launch; sets each layer's ``grad`` to its buffer."""
        if not self.prepare(layers, damping):
            return False
        self.launch()
        for layer, out in zip(layers, self._outs):
            layer.grad = out
        return True


def _ru(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class SplitGroupedPrecondition(GroupedPrecondition):
    """The grouped preconditioning GEMMs on PRE-SPLIT operands
    (csrc/gemm3s.hip): every operand lives in a bf16 hi/lo "split image"
    (zero-padded, ``[2, R, L]``) so the kernel stages tiles global -> LDS by
    LDS-DMA and issues three bf16 MFMAs per fragment pair with no split work:

    * eigenbases / inverses: split once per second-order update (re-split
      when the tensor's address or version changes, i.e. after an in-place
      install);
    * ``[Wg | bg]``: one multi-tensor split launch per step (bias appended);
    * t1, t2, t3: written split by the producing GEMM's epilogue.

    Eigen:   T1 t1 = [Wg|bg] QA, T2 t2 = (QG^T t1) (.) S, T3 t3 = QG t2,
             T4 P = t3 QA^T.   Inverse: T1 t1 = [Wg|bg] A^-1, T3 P = G^-1 t1.
    Same interface as ``GroupedPrecondition`` (tables cached / pinned the
    same way).  Per layer it keeps ~4 split images of the gradient's shape
    plus one of each basis (bf16 x 2 = fp32-sized).
    """

    def __init__(self) -> None:
        super().__init__()
        self._cache = _TableCache(slots_per_entry=6)

    @staticmethod
    def _images(layer: Any, kind: str, g: int, a: int, dev: torch.device) -> dict:
        st = getattr(layer, '_g3s', None)
        key = (kind, g, a, str(dev))
        if st is None or st['key'] != key:
            al = int(native().gemm3s_align())
            gp, ap = _ru(g, al), _ru(a, al)

            def z(r: int, c: int) -> torch.Tensor:
                return torch.zeros(2, r, c, dtype=torch.bfloat16, device=dev)

            st = {'key': key, 'w': z(gp, ap), 't1': z(gp, ap), 'fa': z(ap, ap), 'fg': z(gp, gp),
                  'fa_ver': None, 'fg_ver': None}
            if kind == 'eigen':
                st['t2'] = z(gp, ap)
                st['t3'] = z(gp, ap)
            layer._g3s = st
        return st

    @staticmethod
    def _capturing() -> bool:
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()

    def _resplit(self, todo: list) -> None:
        """Split static operands whose content changed (one launch)."""
        if not todo:
            return
        lib = native()
        srcs = [s for s, _ in todo]
        tab, blocks, _host = lib.build_split_table(srcs, [None] * len(srcs), [d for _, d in todo], None)
        lib.split_pad_multi(tab, len(srcs), blocks)
        self._static_keepalive = (tab, _host, srcs)

    def prepare(self, layers: list, damping: float) -> bool:
        lib = native()
        if lib is None or not layers or not grouped_gemm_enabled():
            return False
        ops = []
        for layer in layers:
            o = self._operands(layer)
            if o is None:
                return False
            ops.append(o)
        split = []
        t = {k: [] for k in ('t1', 't2', 't3e', 't3i', 't4')}
        key: list = [damping]
        todo = []
        outs: list[torch.Tensor] = []
        for layer, (kind, wm, bg, fa, fg) in zip(layers, ops):
            g, a = fg.shape[0], fa.shape[0]
            dev = fa.device
            st = self._images(layer, kind, g, a, dev)
            for name, f in (('fa', fa), ('fg', fg)):
                ver = (f.data_ptr(), f._version)
                if st[name + '_ver'] != ver:
                    todo.append((f if f.stride(1) == 1 else f.contiguous(), st[name]))
                    st[name + '_ver'] = ver
            out = layer.precond_out(dev)
            if tuple(out.shape) != (g, a) or out.stride(1) != 1:
                return False
            outs.append(out)
            split.append((wm, bg, st['w']))
            key.append((kind, id(layer), wm.data_ptr(), None if bg is None else bg.data_ptr(),
                        out.data_ptr(), st['w'].data_ptr()))
            none3 = (None, None, None)
            if kind == 'eigen':
                t['t1'].append((st['w'], st['fa'], st['t1'], none3, (g, a, a)))
                if layer.prediv_eigenvalues:
                    scale = (layer.dgda, None, None)
                else:
                    scale = (None, layer.dg, layer.da)
                key.append((layer.prediv_eigenvalues,) + tuple(
                    None if s is None else s.data_ptr() for s in scale))
                t['t2'].append((st['fg'], st['t1'], st['t2'], scale, (g, a, g)))
                t['t3e'].append((st['fg'], st['t2'], st['t3'], none3, (g, a, g)))
                t['t4'].append((st['t3'], st['fa'], out, none3, (g, a, a)))
            else:
                t['t1'].append((st['w'], st['fa'], st['t1'], none3, (g, a, a)))
                t['t3i'].append((st['fg'], st['t1'], out, none3, (g, a, g)))
        if todo and self._capturing():
            # a basis changed since the last eager step: its split images are
            # refreshed eagerly (never inside a capture); capture the
            # per-layer path this time
            return False
        self._resplit(todo)
        key_t = tuple(key)
        if key_t != self._key:
            tables = self._cache.get(key_t)
            if tables is None:
                # (table name, a_mc, b_mc, out_split)
                flags = [('t1', False, True, True), ('t2', True, True, True),
                         ('t3e', False, True, True), ('t3i', False, True, False),
                         ('t4', False, False, False)]
                slots = self._cache.reserve()
                tables = []
                stab, sblocks, shost = lib.build_split_table(
                    [s[0] for s in split], [s[1] for s in split], [s[2] for s in split], slots[0])
                tables.append(('split', stab, len(split), sblocks, shost))
                for (name, amc, bmc, osplit), slot in zip(flags, slots[1:]):
                    # longest tiles first: a tile's time is its K loop, and
                    # blocks start in table order, so the K = 4608 / 2304
                    # layers' tiles no longer form the launch's tail
                    rows = sorted(t[name], key=lambda r: (-r[4][2], -r[4][0] * r[4][1]))
                    if not rows:
                        continue
                    meta: list[int] = []
                    for r in rows:
                        meta.extend(r[4])
                    sc = [r[3] for r in rows]
                    tab, tiles, host = lib.build_gemm3s_table(
                        [r[0] for r in rows], [r[1] for r in rows], [r[2] for r in rows],
                        [s[0] for s in sc], [s[1] for s in sc], [s[2] for s in sc], meta,
                        [float(damping) if s[1] is not None else 0.0 for s in sc],
                        amc, bmc, osplit, slot)
                    tables.append((name, tab, len(rows), tiles, (amc, bmc, osplit), host))
                self._cache.put(key_t, tables, slots)
            self._tables = tables
            self._key = key_t
        self._layers = layers
        self._outs = outs
        return True

    def launch(self) -> None:
        lib = native()
        for entry in self._tables:
            if entry[0] == 'split':
                _, tab, n, blocks, _ = entry
                lib.split_pad_multi(_used_here(tab), n, blocks)
            else:
                _, tab, n, tiles, (amc, bmc, osplit), _ = entry
                lib.gemm3s_grouped(_used_here(tab), n, tiles, amc, bmc, osplit)


def grouped_gemm_mode() -> str:
    """``KFAC_PRECOND_GEMM``: split (default: pre-split images, LDS-DMA
    staging, csrc/gemm3s.hip), bf16x3 (in-kernel split, csrc/gemm3.hip) or
    torch (per-layer hipBLASLt fp32).  Same box, alternating runs: ResNet-50
    2183 / 2190 vs 2170 / 2172 img/s, GPT-NeoX-125M 246.2k / 247.0k vs
    238.4k / 238.8k tokens/s (profiles/gemm3s_integration_ab_r2.txt)."""
    return getenv('KFAC_PRECOND_GEMM', 'split').lower()


def make_grouped() -> GroupedPrecondition:
    if grouped_gemm_mode() == 'split':
        return SplitGroupedPrecondition()
    return GroupedPrecondition()
