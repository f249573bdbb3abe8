"""K-FAC runtime: hooks, step schedule, KL clip, checkpointing.

Reference: ``kfac/base_preconditioner.py:21-477``.  Public surface and
semantics are the same (hyperparameters as constants or callables of the
step, ``step()`` / ``state_dict()`` / ``load_state_dict()`` /
``memory_usage()`` / ``reset_batch()``, identical collective issue order on
every rank).  MI355X-first differences:

* Hooks.  One forward hook per module computes the A contribution straight
  from the live input (no clone) and registers a tensor hook on the output
  for G (instead of ``register_full_backward_hook``, which wraps every
  output in an extra autograd node).  With one micro-batch per update the
  accumulate + EMA is a single fused SYRK.
* Second order.  All factors this rank owns are decomposed together
  (``ops.linalg.eigh_many``: one-workgroup LDS Jacobi for n <= 128, the
  native Householder tridiagonalisation chains + divide and conquer above
  that, the two-stage solver for large same-size buckets), then broadcasts
  are issued in the reference's (reversed layer, A then G) order.
* No host syncs in ``step()``.  The KL-clip scale is reduced on the device
  (fp64 accumulator) and applied by the gradient-write kernel; the
  reference performs two ``.item()`` syncs per layer per step.
* Phase timing through HIP events (``tracing.phase``) when enabled.
"""
from __future__ import annotations

import logging
import math
import warnings
from collections import defaultdict
from typing import Any
from typing import Callable

import torch

from distributed_kfac_pytorch_amd import tracing
from distributed_kfac_pytorch_amd.graphs import _no_gc
from distributed_kfac_pytorch_amd.layers.base import KFACBaseLayer
from distributed_kfac_pytorch_amd.layers.eigen import KFACEigenLayer
from distributed_kfac_pytorch_amd.layers.inverse import KFACInverseLayer
from distributed_kfac_pytorch_amd.ops import linalg
from distributed_kfac_pytorch_amd.ops import precondition as pops
from distributed_kfac_pytorch_amd.parallel.assignment import WorkAssignment
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size
from distributed_kfac_pytorch_amd.parallel.comm import (
    TorchDistributedCommunicator,
)
from distributed_kfac_pytorch_amd.utils.env import getenv

logger = logging.getLogger(__name__)
# diagnostics only: compute P but leave the raw gradients in place


class StepGraphs:
    """HIP-graph replay of the per-step precondition (+ apply) phases.

    Between second-order updates the precondition phase is a fixed chain of
    ~6 launches per layer (4 hipBLASLt GEMMs, a rank-1 update, the eigenvalue
    scaling) plus the three multi-tensor KL / apply launches -- ~330 small
    launches per ResNet-50 step, host-launch bound from Python.  All operands
    live in persistent buffers (eigenbases are installed in place, P and the
    temporaries are per-layer buffers, gradients are the parameters'
    ``.grad``), so the chain is captured once into a HIP graph and replayed.

    * Without gradient broadcasts (COMM-OPT, one rank): one graph covers
      precondition + KL clip + gradient write.
    * With gradient broadcasts (HYBRID / MEM-OPT): the graph covers this
      rank's preconditioning only; the bucketed RCCL broadcasts and the
      three apply launches follow eagerly.

    Capture happens on the second consecutive eligible step with the same
    buffer addresses and baked-in hyperparameters (damping without prediv);
    any change falls back to eager execution and re-captures.  Inverse-update
    steps always run eagerly.  KL-clip / lr values are read by the kernels
    from a device buffer refreshed before each replay.
    """

    def __init__(self) -> None:
        self.graph: Any = None
        self.key: tuple | None = None
        self.pending_key: tuple | None = None
        self.replays = 0
        self.captures = 0
        self._lane_streams: list = []
        # descriptor tables the current graph reads (pinned in their caches)
        self._held: list[tuple[Any, Any]] = []

    def _release(self) -> None:
        for owner, key in self._held:
            owner.release(key)
        self._held = []

    def _streams(self, n: int) -> list:
        while len(self._lane_streams) < n:
            self._lane_streams.append(torch.cuda.Stream())
        return self._lane_streams[:n]

    @staticmethod
    def _lanes(workers: list) -> list[list]:
        """Split the layers into ``KFAC_PRECOND_STREAMS`` (default 4)
        cost-balanced lanes (greedy LPT on the precondition GEMM flops
        ``g*a*(g+a)``); each lane keeps model order."""
        n = max(1, min(int(getenv('KFAC_PRECOND_STREAMS', '4')), len(workers)))
        if n == 1:
            return [list(workers)]

        def cost(l: Any) -> float:
            g, a = l.module.g_factor_shape[0], l.module.a_factor_shape[0]
            return float(g) * a * (g + a)

        load = [0.0] * n
        which: dict[int, int] = {}
        for i in sorted(range(len(workers)), key=lambda i: -cost(workers[i])):
            k = min(range(n), key=lambda j: load[j])
            load[k] += cost(workers[i])
            which[i] = k
        lanes: list[list] = [[] for _ in range(n)]
        for i, l in enumerate(workers):
            lanes[which[i]].append(l)
        return [ln for ln in lanes if ln]

    @staticmethod
    def _ptr(t: Any) -> int:
        return t.data_ptr() if isinstance(t, torch.Tensor) else 0

    def _key(
        self,
        pre: 'BaseKFACPreconditioner',
        ordered: list,
        bcast: bool,
    ) -> tuple | None:
        parts: list = [bcast]
        for name, layer in ordered:
            worker = pre._assignment.is_grad_worker(name)
            if not worker and not bcast:
                return None
            m = layer.module
            w = m.module.weight.grad
            if w is None or not w.is_cuda:
                return None
            b = m.module.bias.grad if m.has_bias() else None
            parts.append((worker, w.data_ptr(), self._ptr(b), self._ptr(layer._grad_buf)))
            if not worker:
                continue
            if isinstance(layer, KFACEigenLayer):
                if layer.qa is None or layer.qa.dtype != torch.float32:
                    return None
                parts.append((self._ptr(layer.qa), self._ptr(layer.qg),
                              self._ptr(layer.dgda), self._ptr(layer.da),
                              self._ptr(layer.dg), layer.prediv_eigenvalues,
                              self._ptr(layer._tmp1), self._ptr(layer._tmp2)))
            else:
                a_inv = getattr(layer, 'a_inv', None)
                if a_inv is None or a_inv.dtype != torch.float32:
                    return None
                parts.append((self._ptr(a_inv), self._ptr(layer.g_inv),
                              self._ptr(getattr(layer, '_tmp1', None))))
        needs_damping = any(
            isinstance(l, KFACEigenLayer) and not l.prediv_eigenvalues
            for _, l in ordered
        )
        return (tuple(parts), pre.damping if needs_damping else None,
                pre.kl_clip is None)

    def run(
        self,
        pre: 'BaseKFACPreconditioner',
        ordered: list,
        inverse_step: bool,
        skip: set[str] | None = None,
    ) -> bool:
        """Execute the phases through the graph; False = caller runs eager.
        ``skip``: layers already preconditioned during backward (only the
        gradient write covers them)."""
        from distributed_kfac_pytorch_amd.ops import _native

        if inverse_step or not ordered or _native.native() is None:
            self.pending_key = None
            if inverse_step and self.graph is not None:
                # a refresh: capture again afterwards (the refresh may have
                # re-split the bases into new images; a fresh capture costs
                # one eager step per refresh).  The post-refresh corruption of
                # rounds 2-3 was MIOpen's strided 1x1 backward-data reading
                # outside the graph (ops/conv.py), not this phase.
                self.graph = None
                self.key = None
                self._release()
            return False
        if ordered[0][1].module.device.type != 'cuda':
            return False
        if type(pre)._precondition_all is not BaseKFACPreconditioner._precondition_all:
            # a subclass with its own precondition phase (NeoX: gather to the
            # primary, GEMMs, scatter back) -- replaying only the GEMMs would
            # skip the collectives its model-parallel peers enter
            return False
        if torch.cuda.is_current_stream_capturing():
            # inside a whole-step capture (graphs.GraphedTrainStep): the
            # eager launches are recorded into the outer graph
            return False
        bcast = pre._assignment.broadcast_gradients()
        key = self._key(pre, ordered, bcast)
        if key is None:
            return False
        skip = skip or set()
        key = key + (tuple(sorted(skip)),)
        layers = [l for _, l in ordered]
        workers = [l for n, l in ordered
                   if pre._assignment.is_grad_worker(n) and n not in skip]
        if pre._multi_apply is None:
            pre._multi_apply = pops.MultiLayerApply()
        kl = pre.kl_clip
        lr = float(pre.lr)
        if not (key == self.key and self.graph is not None):
            if key != self.pending_key:
                # first sighting of this configuration: run eagerly, capture next
                self.pending_key = key
                return False
            if not bcast and not pre._multi_apply.prepare(layers, kl, lr, use_buffers=True):
                return False
            damping = pre.damping
            if pre._grouped is None:
                pre._grouped = pops.make_grouped()
            # grouped MFMA GEMMs (4 launches for all layers); tables are built
            # here, outside the capture
            grouped = pre._grouped.prepare(workers, damping)
            # the graph keeps reading these device tables: pin them so the
            # table caches never evict (free) them while the graph lives
            self.graph = None
            self._release()
            if grouped:
                self._held.append((pre._grouped, pre._grouped.hold()))
            if not bcast:
                self._held.append((pre._multi_apply, pre._multi_apply.hold()))
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            lanes = [] if grouped else self._lanes(workers)
            with _no_gc(), torch.cuda.stream(side):
                # thread_local: only this thread is barred from unsafe HIP
                # calls while capturing -- RCCL's watchdog thread keeps
                # querying its events (multi-rank jobs); no GC: a collected
                # cycle holding an old graph would destroy it mid-capture
                with torch.cuda.graph(g, stream=side, capture_error_mode='thread_local'):
                    if grouped:
                        pre._grouped.launch()
                    # otherwise fork: independent per-layer GEMM chains run as
                    # parallel graph branches (small layers cannot fill 256
                    # CUs alone)
                    for lane, members in zip(self._streams(len(lanes)), lanes):
                        lane.wait_stream(side)
                        with torch.cuda.stream(lane):
                            for l in members:
                                l.preconditioned_grad(damping=damping)
                    for lane in self._streams(len(lanes)):
                        side.wait_stream(lane)
                    if not bcast:
                        pre._multi_apply.launch(kl is not None)
            torch.cuda.current_stream().wait_stream(side)
            # descriptor tables built during the capture: one eager upload
            _native.flush_table_uploads()
            self.graph, self.key, self.pending_key = g, key, None
            self.captures += 1
        elif not bcast and not pre._multi_apply.prepare(layers, kl, lr, use_buffers=True):
            return False
        label = 'precondition(graph)' if bcast else 'precondition+apply(graph)'
        with tracing.phase(label):
            self.graph.replay()
        self.replays += 1
        if not bcast:
            for l in layers:
                l.grad = None
            return True
        for l in workers:
            l.grad = l._grad_buf
        with tracing.phase('grad_broadcast'):
            for name, l in ordered:
                l.broadcast_grad(
                    src=pre._assignment.src_grad_worker(name),
                    group=pre._assignment.grad_receiver_group(name),
                    bucketed=True,
                )
            pre._tdc.flush_broadcast_buckets()
            pre._tdc.flush_allreduce_buckets()
        with tracing.phase('apply'):
            pre._apply_gradients(ordered, kl)
        return True

def _batchable_inverse(layer: KFACBaseLayer) -> bool:
    """Plain INVERSE-method layers with symmetric factors are inverted by
    ``ops.linalg.inverse_many``; subclasses that override ``compute_*_inv``
    (e.g. the diagonal-A embedding layer) keep their own path."""
    return (
        isinstance(layer, KFACInverseLayer)
        and getattr(layer.compute_a_inv, '__func__', None) is KFACInverseLayer.compute_a_inv
        and getattr(layer.compute_g_inv, '__func__', None) is KFACInverseLayer.compute_g_inv
        and layer.symmetric_factors
    )


class BaseKFACPreconditioner:
    """Distributed K-FAC gradient preconditioner (layer-agnostic runtime)."""

    def __init__(
        self,
        layers: dict[torch.nn.Module, tuple[str, KFACBaseLayer]],
        *,
        assignment: WorkAssignment,
        tdc: TorchDistributedCommunicator,
        factor_update_steps: Callable[[int], int] | int = 1,
        inv_update_steps: Callable[[int], int] | int = 1,
        damping: Callable[[int], float] | float = 0.001,
        factor_decay: Callable[[int], float] | float = 0.95,
        kl_clip: Callable[[int], float] | float | None = 0.001,
        lr: Callable[[int], float] | float = 0.1,
        accumulation_steps: int = 1,
        update_factors_in_hook: bool = True,
        defaults: dict[str, Any] | None = None,
        loglevel: int = logging.DEBUG,
    ) -> None:
        """Init BaseKFACPreconditioner.

        Args:
            layers: ``{module: (name, KFAC layer)}`` in model order.
            assignment: work placement built for ``layers``.
            tdc: shared communicator.
            factor_update_steps: steps between factor updates (or callable).
            inv_update_steps: steps between second-order updates (or callable).
            damping: Tikhonov damping (or callable).
            factor_decay: running-average weight of the factors (or callable).
            kl_clip: KL-clip parameter (or callable); ``None`` disables the
                clip (the reference documents this but raises on it,
                SURVEY 5.10 #1 -- fixed here).
            lr: learning rate used by the KL clip (or callable).
            accumulation_steps: forward/backward passes per optimizer step.
            update_factors_in_hook: update running factors and start their
                all-reduce inside the hooks (else at the start of ``step``).
            defaults: extra key/values shown in ``repr``.
            loglevel: logging level of registration / assignment messages.
        """
        if not callable(factor_update_steps) and not 0 < factor_update_steps:
            raise ValueError('factor_update_steps must be > 0')
        if not callable(inv_update_steps) and not 0 < inv_update_steps:
            raise ValueError('inv_update_steps must be > 0')
        if not callable(damping) and not 0.0 < damping:
            raise ValueError('damping must be > 0')
        if not callable(factor_decay) and not 0.0 < factor_decay <= 1:
            raise ValueError('factor_decay must be in (0, 1]')
        if kl_clip is not None and not callable(kl_clip) and not 0.0 < kl_clip:
            raise ValueError('kl_clip must be > 0')
        if not callable(lr) and not 0.0 <= lr:
            raise ValueError('lr be > 0')
        if not 0 < accumulation_steps:
            raise ValueError('accumulation_steps must be > 0')
        if (
            not callable(inv_update_steps)
            and not callable(factor_update_steps)
            and inv_update_steps % factor_update_steps != 0
        ):
            warnings.warn(
                'It is suggested that inv_update_steps be an integer multiple '
                'of factor_update_steps',
            )
        self._accumulation_steps = accumulation_steps
        self._assignment = assignment
        self._damping = damping
        self._defaults = defaults
        self._factor_decay = factor_decay
        self._factor_update_steps = factor_update_steps
        self._inv_update_steps = inv_update_steps
        self._kl_clip = kl_clip
        self._layers = layers
        self._loglevel = loglevel
        self._lr = lr
        self._tdc = tdc
        self._update_factors_in_hook = update_factors_in_hook
        self._steps = 0
        self._mini_steps: dict[str, int] = defaultdict(int)
        # backward-hook count per layer, kept apart from the forward count so
        # a schedule that runs several forwards before their backwards (a
        # GPipe / 1F1B pipeline) still folds G exactly once per step; with
        # interleaved forward / backward it equals the reference's shared
        # counter (kfac/base_preconditioner.py:_save_grad_output)
        self._mini_steps_g: dict[str, int] = defaultdict(int)
        self._kl_acc: torch.Tensor | None = None
        self._kl_scale: torch.Tensor | None = None
        self._multi_apply: Any = None
        self._grouped: Any = None
        self._graphs: Any = None
        # Precondition-phase HIP graphs (StepGraphs) are opt-in
        # (KFAC_GRAPHS=1): on the eager step path -- every multi-rank job --
        # replaying them left the GPU idle ~7 ms per ResNet-50 step (eager
        # plain step 24.4-25.1 ms with them vs 17.06 ms without, fp32, same
        # tree: profiles/r5/eager_stepgraphs/), while the grouped kernels
        # launched eagerly are only 4 + 3 launches.  Whole-step graphs
        # (graphs.GraphedTrainStep) capture the phase anyway.
        if getenv('KFAC_GRAPHS', '0') == '1':
            self._graphs = StepGraphs()
        # factor SYRKs (+ their all-reduce) run on a side stream forked from
        # the hook's stream, so they overlap the rest of forward / backward;
        # joined back before anything reads the factors (KFAC_FACTOR_STREAM=0:
        # inline)
        self._factor_streams: dict[Any, torch.cuda.Stream] = {}
        self._factor_forked: set = set()
        # per device: event on the factor stream after the latest A-factor
        # (forward hook) work -- step() waits only for that part when the
        # G-factor work may finish lazily (_lazy_factor_join)
        self._factor_a_events: dict[Any, torch.cuda.Event] = {}
        self._factor_inputs: list[tuple[torch.Tensor, int]] = []
        self._factor_stream_off = False
        # Hook work queued for the side stream and launched a segment at a
        # time (_flush_factor_segment): one stream fork / event / context
        # switch per KFAC_FACTOR_SEGMENT layers instead of per layer (the
        # per-hook stream switching was ~40 % of the eager factor step's
        # host issue: profiles/r5/host_env/host_profile_factor.txt).  A
        # pass's last layer (forward: the last registered, backward: the
        # first) and every reader of the factors flush what is queued.
        self._factor_pending: list[tuple[torch.Tensor, Callable[[], None], str, int]] = []
        self._factor_segment = max(1, int(getenv('KFAC_FACTOR_SEGMENT', '8')))
        self._layer_index = {m: i for i, m in enumerate(self._layers)}
        self._hook_handles: list[Any] = []
        for module in self._layers:
            self._hook_handles.append(
                module.register_forward_hook(self._forward_hook),
            )
        # early preconditioning (set up at the first step, _setup_early)
        self._early: dict[str, Any] | None = None
        # packed factor buffers are laid out once, before the first factor
        # update (_plan_packed)
        self._packed_planned = False

    # ----------------------------------------------------------------- repr
    def __repr__(self) -> str:
        params: list[tuple[str, Any]] = [
            ('accumulation_steps', self._accumulation_steps),
            ('assignment', self._assignment.__class__.__name__),
            ('damping', self._damping),
            ('factor_decay', self._factor_decay),
            ('factor_update_steps', self._factor_update_steps),
            ('inv_update_steps', self._inv_update_steps),
            ('kl_clip', self._kl_clip),
            ('layers', len(self._layers)),
            ('loglevel', self._loglevel),
            ('lr', self._lr),
            ('steps', self.steps),
            ('update_factors_in_hook', self._update_factors_in_hook),
        ]
        if self._defaults is not None:
            params.extend(self._defaults.items())
        body = '\n'.join(f'  {k}={v},' for k, v in sorted(params, key=lambda x: x[0]))
        return f'{self.__class__.__name__}(\n{body}\n)'

    # ------------------------------------------------------- hyperparameters
    def _value(self, v: Any) -> Any:
        return v(self.steps) if callable(v) else v

    @property
    def damping(self) -> float:
        return self._value(self._damping)

    @property
    def factor_decay(self) -> float:
        return self._value(self._factor_decay)

    @property
    def kl_clip(self) -> float | None:
        return self._value(self._kl_clip)

    @property
    def lr(self) -> float:
        return self._value(self._lr)

    @property
    def factor_update_steps(self) -> int:
        return self._value(self._factor_update_steps)

    @property
    def inv_update_steps(self) -> int:
        return self._value(self._inv_update_steps)

    @property
    def steps(self) -> int:
        return self._steps

    # ------------------------------------------------------------ checkpoint
    def state_dict(self, include_factors: bool = True) -> dict[str, Any]:
        """Reference-format state: steps, non-callable hyperparameters and
        (optionally) ``{'layers': {name: {'A': .., 'G': ..}}}``."""
        self._join_factor_streams()
        sd: dict[str, Any] = {'steps': self.steps}
        for key in (
            'factor_update_steps',
            'inv_update_steps',
            'damping',
            'factor_decay',
            'kl_clip',
            'lr',
        ):
            v = getattr(self, f'_{key}')
            if not callable(v):
                sd[key] = v
        if include_factors:
            sd['layers'] = {
                name: layer.state_dict() for name, layer in self._layers.values()
            }
        return sd

    def load_state_dict(
        self,
        state_dict: dict[str, Any],
        compute_inverses: bool = True,
    ) -> None:
        """Restore ``state_dict``; optionally recompute (and broadcast) all
        second-order state from the loaded factors."""
        self._join_factor_streams()
        self._steps = state_dict['steps']
        for key in (
            'factor_update_steps',
            'inv_update_steps',
            'damping',
            'factor_decay',
            'kl_clip',
            'lr',
        ):
            if key in state_dict:
                setattr(self, f'_{key}', state_dict[key])
        if 'layers' in state_dict:
            if len(state_dict['layers']) != len(self._layers):
                raise ValueError(
                    'loaded state dict contains a different number of layers',
                )
            by_name = {name: layer for name, layer in self._layers.values()}
            for name, layer_state in state_dict['layers'].items():
                if name in by_name:
                    by_name[name].load_state_dict(layer_state)
        elif compute_inverses:
            warnings.warn(
                'Layer factors are not included in the state_dict so '
                'inverses cannot be computed. Skipping inverse computation.',
            )
            compute_inverses = False
        if compute_inverses:
            items = list(self._layers.values())
            self._compute_second_order(items, all_ranks=True)
            if self._assignment.broadcast_inverses():
                for name, layer in items:
                    layer.broadcast_a_inv(
                        src=self._assignment.inv_worker(name, 'A'),
                        group=self._assignment.grad_worker_group(name),
                    )
                    layer.broadcast_g_inv(
                        src=self._assignment.inv_worker(name, 'G'),
                        group=self._assignment.grad_worker_group(name),
                    )

    # ------------------------------------------------------------------ step
    def _compute_second_order(
        self,
        items: list[tuple[str, KFACBaseLayer]],
        all_ranks: bool = False,
    ) -> None:
        """Decompose / invert every factor this rank owns, batched."""
        rank = get_rank()
        damping = self.damping
        mine_a = [
            (n, l) for n, l in items
            if all_ranks or rank == self._assignment.inv_worker(n, 'A')
        ]
        mine_g = [
            (n, l) for n, l in items
            if all_ranks or rank == self._assignment.inv_worker(n, 'G')
        ]
        def batchable(l: KFACBaseLayer) -> bool:
            return (
                isinstance(l, KFACEigenLayer)
                and l.symmetric_factors
                and getattr(l, 'supports_batched_eigh', True)
            )

        eig_a = [(n, l) for n, l in mine_a if batchable(l)]
        eig_g = [(n, l) for n, l in mine_g if batchable(l)]
        batched = {id(l) for _, l in eig_a} | {id(l) for _, l in eig_g}
        mats = []
        for _, l in eig_a:
            if l.a_factor is None:
                raise RuntimeError('Cannot eigendecompose A before A has been computed')
            mats.append(l.a_factor)
        for _, l in eig_g:
            if l.g_factor is None:
                raise RuntimeError('Cannot eigendecompose G before G has been computed')
            mats.append(l.g_factor)
        results = linalg.eigh_many(mats) if mats else []
        for (_, l), (d, q) in zip(eig_a, results[: len(eig_a)]):
            assert isinstance(l, KFACEigenLayer)
            l.set_a_eig(d, q)
        for (_, l), (d, q) in zip(eig_g, results[len(eig_a):]):
            assert isinstance(l, KFACEigenLayer)
            l.set_g_eig(d, q, damping)
        # INVERSE method: every owned symmetric factor in one batched call
        inv_a = [(n, l) for n, l in mine_a if _batchable_inverse(l)]
        inv_g = [(n, l) for n, l in mine_g if _batchable_inverse(l)]
        mats = []
        for _, l in inv_a:
            if l.a_factor is None:
                raise RuntimeError('Cannot invert A before A has been computed')
            mats.append(l.a_factor)
        for _, l in inv_g:
            if l.g_factor is None:
                raise RuntimeError('Cannot invert G before G has been computed')
            mats.append(l.g_factor)
        invs = linalg.inverse_many(mats, damping) if mats else []
        for (_, l), x in zip(inv_a, invs[: len(inv_a)]):
            l.set_a_inv(x)
        for (_, l), x in zip(inv_g, invs[len(inv_a):]):
            l.set_g_inv(x)
        batched |= {id(l) for _, l in inv_a} | {id(l) for _, l in inv_g}
        for _, l in mine_a:
            if id(l) not in batched:
                l.compute_a_inv(damping=damping)
        for _, l in mine_g:
            if id(l) not in batched:
                l.compute_g_inv(damping=damping)

    @staticmethod
    def _bcast_inv(fn: Callable[..., None], src: int, group: Any) -> None:
        fn(src=src, group=group, bucketed=True)

    def _lazy_factor_join(self) -> bool:
        """May this ``step()`` leave the G-factor SYRKs of the backward hooks
        running on the factor stream (``KFAC_FACTOR_JOIN``, default
        ``lazy``; ``full`` joins every step as before)?

        Nothing in a step that does not refresh the second-order state reads
        the factors: preconditioning uses the eigenbases (or inverses), the
        KL clip and the optimizer the gradients.  The G SYRKs read only
        autograd's output gradients (kept alive for the side stream by
        ``record_stream``), so they can finish under the preconditioning, the
        optimizer step and the next forward instead of extending the
        factor-update step.  The A SYRKs read the layer inputs -- tensors the
        caller may overwrite in place after the step (the input batch) -- so
        they are always waited for (``_sync_factor_inputs``).  Every reader of
        the factors joins first: second-order updates, checkpoints,
        ``memory_usage``, graph capture.  Single process only: with a process
        group the buckets / packed chunks still unlaunched at ``step()`` are
        all-reduced from the compute stream and need the full join."""
        if getenv('KFAC_FACTOR_JOIN', 'lazy') != 'lazy':
            return False
        if self.steps % self.inv_update_steps == 0:
            return False
        if not self._update_factors_in_hook or self._accumulation_steps != 1:
            return False
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return False  # a captured step joins every stream it forked
        return get_world_size() == 1 and self._graphs is None

    def _sync_factor_inputs(self) -> None:
        """Partial join: the current stream waits for the A-factor work only
        (the G SYRKs keep running on the side stream); the inputs' in-place
        modification check runs as in ``_join_factor_streams``."""
        if self._factor_pending:
            self._flush_factor_segment()
        for dev in self._factor_forked:
            ev = self._factor_a_events.get(dev)
            if ev is not None:
                torch.cuda.current_stream(dev).wait_event(ev)
        self._check_factor_inputs()

    def sync_factors(self) -> None:
        """Order the current stream after every pending factor update (the
        lazy G-factor SYRKs included)."""
        self._join_factor_streams()

    @torch.no_grad()
    def step(self) -> None:
        """One K-FAC step: call after ``loss.backward()`` (gradients already
        averaged by DDP) and before ``optimizer.step()``."""
        if self._lazy_factor_join():
            self._sync_factor_inputs()
        else:
            self._join_factor_streams()
        ordered = list(reversed(list(self._layers.values())))
        if (
            not self._update_factors_in_hook
            and self.steps % self.factor_update_steps == 0
        ):
            self._plan_packed()
            with tracing.phase('factor_update'):
                decay = self.factor_decay
                for name, layer in ordered:
                    self._mini_steps[name] = 0
                    self._mini_steps_g[name] = 0
                    layer.update_a_factor(alpha=decay)
                    layer.reduce_a_factor(self._assignment.factor_group(name, 'A'))
                    layer.update_g_factor(alpha=decay)
                    layer.reduce_g_factor(self._assignment.factor_group(name, 'G'))
        self._tdc.flush_allreduce_buckets()

        if self.steps % self.inv_update_steps == 0:
            with tracing.phase('inverse'):
                self._compute_second_order(ordered)
            if self._assignment.broadcast_inverses():
                with tracing.phase('inverse_broadcast'):
                    # fused per (column group, source) buckets: a handful of
                    # RCCL broadcasts instead of ~4 per layer
                    for name, layer in ordered:
                        if self._assignment.is_grad_worker(name):
                            self._bcast_inv(layer.broadcast_a_inv,
                                            self._assignment.inv_worker(name, 'A'),
                                            self._assignment.grad_worker_group(name))
                            self._bcast_inv(layer.broadcast_g_inv,
                                            self._assignment.inv_worker(name, 'G'),
                                            self._assignment.grad_worker_group(name))
                    self._tdc.flush_broadcast_buckets()
            self._tdc.flush_allreduce_buckets()
            # eigenbases changed: refresh their bf16 hi/lo planes for the
            # grouped GEMMs now, eagerly (never inside a later graph capture)
            if pops.presplit_enabled():
                for name, layer in ordered:
                    if isinstance(layer, KFACEigenLayer) and self._assignment.is_grad_worker(name):
                        layer.q_split()

        inverse_step = self.steps % self.inv_update_steps == 0
        if self._early is None:
            self._setup_early(ordered)
        early = self._join_early()
        if self._graphs is None or not self._graphs.run(self, ordered, inverse_step, early):
            with tracing.phase('precondition'):
                if early:
                    self._precondition_all(ordered, skip=early)
                else:
                    self._precondition_all(ordered)
            with tracing.phase('apply'):
                self._apply_gradients(ordered, self.kl_clip)

        self._steps += 1
        self._mini_steps = defaultdict(int)
        self._mini_steps_g = defaultdict(int)

    # ------------------------------------------------ early preconditioning
    def _setup_early(self, ordered: list[tuple[str, KFACBaseLayer]]) -> None:
        """Choose the layers preconditioned during backward (once).

        Backward produces the last layers' gradients first; their grouped
        preconditioning GEMMs (the bulk of the per-step K-FAC work: ResNet-50's
        layer4 + fc hold ~60 % of the flops) need nothing else from the step,
        so they are launched on a side stream as soon as every gradient of
        the group has been accumulated and run while backward continues
        through the earlier layers (small-batch convolutions leave most of
        the MFMA capacity idle).  The rest run in ``step()`` as before.

        Only for single-process CUDA jobs without gradient accumulation or
        gradient broadcasts: with DDP the gradient is final only after its
        bucket's all-reduce.  ``KFAC_PRECOND_OVERLAP=0`` disables it;
        ``KFAC_PRECOND_OVERLAP_FRAC`` (0.5) is the share of the flops
        ``g*a*(g+a)`` moved into the early group.  Never on second-order
        update steps (the bases change in ``step()``)."""
        self._early = {'names': [], 'count': 0, 'total': 0, 'pending': False}
        if getenv('KFAC_PRECOND_OVERLAP', '0') == '0':
            return
        if self._accumulation_steps != 1 or get_world_size() > 1:
            return
        if any(getattr(l, '_scaler', None) is not None for _, l in ordered):
            return  # a GradScaler unscales the gradients after backward
        if type(self)._precondition_all is not BaseKFACPreconditioner._precondition_all:
            return  # a subclass with its own precondition phase (NeoX)
        if self._assignment.broadcast_gradients() or not pops.grouped_gemm_enabled():
            return
        workers = [(n, l) for n, l in ordered if self._assignment.is_grad_worker(n)]
        if len(workers) < 2 or workers[0][1].module.device.type != 'cuda':
            return

        def cost(l: KFACBaseLayer) -> float:
            g, a = l.module.g_factor_shape[0], l.module.a_factor_shape[0]
            return float(g) * a * (g + a)

        frac = float(getenv('KFAC_PRECOND_OVERLAP_FRAC', '0.5'))
        total = sum(cost(l) for _, l in workers)
        names, acc = [], 0.0
        for n, l in workers[:-1]:
            if acc >= frac * total:
                break
            names.append(n)
            acc += cost(l)
        params = []
        for n, l in workers:
            if n in names:
                params.append(l.module.module.weight)
                if l.module.has_bias():
                    params.append(l.module.module.bias)
        if not names or any(not p.requires_grad for p in params):
            return
        for p in params:
            self._hook_handles.append(p.register_post_accumulate_grad_hook(self._early_ready))
        self._early.update(
            names=names, total=len(params), grouped=pops.make_grouped(), params=params,
            layers=[l for n, l in workers if n in names],
            stream=torch.cuda.Stream(device=workers[0][1].module.device),
        )

    def _early_ready(self, param: torch.Tensor) -> None:
        st = self._early
        if st is None or not st['names']:
            return
        st['count'] += 1
        if st['count'] != st['total'] or self.steps % self.inv_update_steps == 0:
            return
        side = st['stream']
        side.wait_stream(torch.cuda.current_stream(side.device))
        # the side stream reads the gradients now: anything that changes them
        # before step() (GradScaler.unscale_, clip_grad_norm_) bumps their
        # version, and _join_early then redoes those layers eagerly
        st['versions'] = [g._version for g in (p.grad for p in st['params']) if g is not None]
        with torch.cuda.stream(side):
            st['pending'] = bool(st['grouped'].run(st['layers'], self.damping))

    def _join_early(self) -> set[str]:
        """Names preconditioned during this step's backward (side stream
        joined into the current stream); resets the per-step count."""
        st = self._early
        if st is None:
            return set()
        done = set(st['names']) if st['pending'] else set()
        if st['pending']:
            torch.cuda.current_stream(st['stream'].device).wait_stream(st['stream'])
            now = [g._version for g in (p.grad for p in st['params']) if g is not None]
            if now != st.get('versions'):
                # a gradient changed after the early launch (unscale / clip):
                # the early P is stale, precondition those layers again
                done = set()
        st['pending'] = False
        st['count'] = 0
        return done

    def _precondition_all(self, ordered: list[tuple[str, KFACBaseLayer]],
                          skip: set[str] | None = None) -> None:
        """Precondition this rank's layers (except ``skip``: already done
        during backward); broadcast results if needed."""
        damping = self.damping
        bcast = self._assignment.broadcast_gradients()
        skip = skip or set()
        workers = [l for n, l in ordered
                   if self._assignment.is_grad_worker(n) and n not in skip]
        grouped = False
        if workers and workers[0].module.device.type == 'cuda':
            if self._grouped is None:
                self._grouped = pops.make_grouped()
            grouped = self._grouped.run(workers, damping)
        for name, layer in ordered:
            if not grouped and self._assignment.is_grad_worker(name) and name not in skip:
                layer.preconditioned_grad(damping=damping)
            if bcast:
                layer.broadcast_grad(
                    src=self._assignment.src_grad_worker(name),
                    group=self._assignment.grad_receiver_group(name),
                    bucketed=True,
                )
        self._tdc.flush_broadcast_buckets()
        self._tdc.flush_allreduce_buckets()

    def _apply_gradients(
        self,
        ordered: list[tuple[str, KFACBaseLayer]],
        kl: float | None,
    ) -> None:
        """KL-clip scale + in-place gradient write for every layer.

        GPU fast path: three multi-tensor launches for the whole model
        (``ops.precondition.MultiLayerApply``); otherwise per layer.
        """
        if not ordered:
            return
        if self._multi_apply is None:
            self._multi_apply = pops.MultiLayerApply()
        if self._multi_apply.run(
            [layer for _, layer in ordered],
            kl,
            float(self.lr) if kl is not None else 0.0,
        ):
            return
        scale = None if kl is None else self._device_grad_scale(ordered, kl)
        for _, layer in ordered:
            layer.update_grad(scale=scale)

    def _kl_buffers(self, device: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
        if self._kl_acc is None or self._kl_acc.device != device:
            self._kl_acc = torch.zeros(1, dtype=torch.float64, device=device)
            self._kl_scale = torch.ones(1, dtype=torch.float32, device=device)
        assert self._kl_scale is not None
        return self._kl_acc, self._kl_scale

    def _device_grad_scale(
        self,
        ordered: list[tuple[str, KFACBaseLayer]],
        kl_clip: float,
    ) -> torch.Tensor | float:
        """KL-clip scale as a 1-element device tensor (no host sync)."""
        if not ordered:
            return 1.0
        acc, scale = self._kl_buffers(ordered[0][1].module.device)
        for _, layer in ordered:
            p = layer.grad
            if p is None:
                raise AssertionError('layer gradient has not been preconditioned')
            wg = layer.module.weight_grad_matrix()
            bg = layer.module.get_bias_grad() if layer.module.has_bias() else None
            pops.kl_dot_(p, wg, bg, acc)
        pops.kl_finalize(acc, scale, float(kl_clip), float(self.lr))
        return scale

    def _compute_grad_scale(self) -> float:
        """KL-clip scale as a Python float (reference API; syncs once)."""
        layers = list(reversed(list(self._layers.values())))
        if not layers:
            return 1.0
        vg = 0.0
        lr2 = self.lr ** 2
        for _, layer in layers:
            if layer.grad is None:
                raise AssertionError('layer gradient has not been preconditioned')
            p = layer.grad.to(torch.float64)
            wg = layer.module.weight_grad_matrix().to(torch.float64)
            if layer.module.has_bias():
                bg = layer.module.get_bias_grad().reshape(-1, 1).to(torch.float64)
                vg += float((p[:, :-1] * wg).sum() + (p[:, -1:] * bg).sum()) * lr2
            else:
                vg += float((p * wg).sum()) * lr2
        if vg == 0.0:
            return 1.0
        return min(1.0, math.sqrt(self.kl_clip / abs(vg)))

    def reset_batch(self) -> None:
        """Drop accumulated (not yet folded) factor contributions."""
        self._join_factor_streams()
        for _, layer in self._layers.values():
            layer.reset_batch()

    def memory_usage(self) -> dict[str, int]:
        """Bytes held by K-FAC state on this rank, per category + total."""
        self._join_factor_streams()
        self._tdc.flush_allreduce_buckets()
        sizes: dict[str, int] = defaultdict(int)
        for _, layer in self._layers.values():
            for k, v in layer.memory_usage().items():
                sizes[k] += v
        sizes['total'] = sum(sizes.values())
        return sizes

    def _plan_packed(self) -> None:
        """Reserve every packed factor slot in hook order -- A factors in
        forward (registration) order, then G factors in backward order -- so
        each group's ``PackedFactorBuffer`` is allocated once at its final
        size and its chunks complete (and launch from the hooks) in the order
        the hooks fill them."""
        if self._packed_planned:
            return
        self._packed_planned = True
        layers = list(self._layers.values())
        order = [(n, l, 'A') for n, l in layers] + [(n, l, 'G') for n, l in reversed(layers)]
        plans: dict[Any, list] = {}
        for name, layer, which in order:
            group = self._assignment.factor_group(name, which)
            if not layer._packed_ok(group):
                continue
            shape = layer.module.a_factor_shape if which == 'A' else layer.module.g_factor_shape
            d = int(shape[0])
            key = (group, torch.float32, layer.module.device)
            plans.setdefault(key, []).append(((id(layer), which), d * (d + 1) // 2))
        for (group, dtype, device), layout in plans.items():
            self._tdc.packed_buffer(group, dtype, device).reserve(layout, dtype, device)

    # ----------------------------------------------------------------- hooks
    def _forward_hook(
        self,
        module: torch.nn.Module,
        inputs: tuple[torch.Tensor, ...],
        output: torch.Tensor,
    ) -> None:
        self._save_input(module, inputs)
        if (
            module.training
            and isinstance(output, torch.Tensor)
            and output.requires_grad
            and torch.is_grad_enabled()
            and self.steps % self.factor_update_steps == 0
        ):
            output.register_hook(
                lambda g, m=module: self._save_grad_output(m, None, (g,)),
            )

    @staticmethod
    def _stream_friendly_backend() -> bool:
        """Collectives that stay device-side: RCCL ('nccl') orders its
        all-reduce after the issuing (side) stream with a HIP event, so the
        factor SYRKs and the all-reduce of every packed-factor chunk they
        complete (launched from the hook, ``PackedFactorBuffer.mark``)
        overlap the rest of forward / backward.  gloo
        stages GPU tensors through the host: there the side stream only adds
        host round trips (2-rank gloo rehearsal on one GPU: factor phases
        65-236 ms/step against <1 ms inline,
        profiles/fstream_w2_ab_mi355x.jsonl), so it stays inline."""
        if get_world_size() <= 1:
            return True
        try:
            import torch.distributed as dist

            return dist.get_backend() == 'nccl'
        except (RuntimeError, ValueError):
            return False

    def _factor_stream(self, t: torch.Tensor) -> torch.cuda.Stream | None:
        # KFAC_FACTOR_STREAM: 1 force on, 0 force off, unset = on for
        # single-process jobs and RCCL process groups
        mode = getenv('KFAC_FACTOR_STREAM', 'auto')
        if not t.is_cuda or self._factor_stream_off or mode == '0':
            return None
        if mode != '1' and not self._stream_friendly_backend():
            return None
        dev = t.device
        s = self._factor_streams.get(dev)
        if s is None:
            s = torch.cuda.Stream(device=dev)
            self._factor_streams[dev] = s
        return s

    def _join_factor_streams(self) -> None:
        """Make the current stream wait for the factor side streams (every
        reader of the factors calls this first)."""
        if self._factor_pending:
            self._flush_factor_segment()
        if not self._factor_forked:
            return
        for dev in self._factor_forked:
            torch.cuda.current_stream(dev).wait_stream(self._factor_streams[dev])
        self._factor_forked = set()
        self._check_factor_inputs()

    def _check_factor_inputs(self) -> None:
        # the side stream read each layer input / output gradient after the
        # hook returned: if the model modified one in place meanwhile (the
        # hazard the reference's input clone guards against), that factor
        # contribution may be stale -- say so and go back to inline updates
        changed = [t for t, v in self._factor_inputs if t._version != v]
        self._factor_inputs = []
        if changed and not self._factor_stream_off:
            self._factor_stream_off = True
            warnings.warn(
                'a K-FAC layer input was modified in place after its forward '
                'hook; factor updates now run inline on the compute stream '
                '(KFAC_FACTOR_STREAM=0 avoids the side stream from the start)',
                stacklevel=2,
            )

    def _on_factor_stream(self, t: torch.Tensor, fn: Callable[[], None],
                          which: str = 'G', last: bool = False) -> None:
        """Run ``fn`` (SYRK + EMA + all-reduce issue of one factor) on the
        side stream after the work that produced ``t``.

        The work is queued and launched with the rest of its segment
        (``_flush_factor_segment``): ``t`` stays referenced by the queue
        until then, and by the caching allocator's stream record after.
        ``last``: the pass's final hook -- flush now."""
        if self._factor_pending and self._factor_pending[-1][2] != which:
            self._flush_factor_segment()  # forward -> backward: A work goes first
        if self._factor_stream(t) is None:
            fn()
            return
        self._factor_pending.append((t, fn, which, t._version))
        if last or len(self._factor_pending) >= self._factor_segment:
            self._flush_factor_segment()

    def _flush_factor_segment(self) -> None:
        """Launch the queued hook work on the side stream: one fork after
        everything the compute stream has issued so far (which produced
        every queued tensor), the layers' SYRKs in hook order, one A event."""
        pending, self._factor_pending = self._factor_pending, []
        if not pending:
            return
        dev = pending[0][0].device
        s = self._factor_stream(pending[0][0])
        if s is None:  # the side stream was switched off meanwhile: inline
            for _, fn, _, _ in pending:
                fn()
            return
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _, fn, _, _ in pending:
                fn()
        if any(w == 'A' for _, _, w, _ in pending):
            ev = self._factor_a_events.get(dev)
            if ev is None:
                ev = self._factor_a_events[dev] = torch.cuda.Event()
            ev.record(s)
        for t, _, _, v in pending:
            t.record_stream(s)
            self._factor_inputs.append((t, v))
        self._factor_forked.add(dev)

    @torch.no_grad()
    def _save_input(self, module: torch.nn.Module, input: tuple[torch.Tensor, ...]) -> None:
        """Forward-hook body: A contribution (+ fused EMA and all-reduce)."""
        if not module.training:
            return
        if self.steps % self.factor_update_steps != 0:
            return
        if not self._packed_planned:
            self._plan_packed()
        name, layer = self._layers[module]
        self._mini_steps[name] += 1
        in_hook = (
            self._update_factors_in_hook
            and self._mini_steps[name] % self._accumulation_steps == 0
        )
        if in_hook and self._accumulation_steps == 1 and isinstance(input[0], torch.Tensor):
            decay = self.factor_decay
            group = self._assignment.factor_group(name, 'A')

            def work() -> None:
                with tracing.phase('factor_a'):
                    layer.save_and_update_a(list(input), alpha=decay)
                layer.reduce_a_factor(group)
            self._on_factor_stream(input[0], work, 'A',
                                   last=self._layer_index[module] == len(self._layers) - 1)
            return
        self._join_factor_streams()
        with tracing.phase('factor_a'):
            if in_hook and self._accumulation_steps == 1:
                layer.save_and_update_a(list(input), alpha=self.factor_decay)
            else:
                layer.save_layer_input(list(input))
                if in_hook:
                    layer.update_a_factor(alpha=self.factor_decay)
        if in_hook:
            layer.reduce_a_factor(self._assignment.factor_group(name, 'A'))

    @torch.no_grad()
    def _save_grad_output(
        self,
        module: torch.nn.Module,
        grad_input: Any,
        grad_output: tuple[torch.Tensor, ...] | torch.Tensor,
    ) -> None:
        """Backward-hook body: G contribution (+ fused EMA and all-reduce)."""
        if not module.training:
            return
        if self.steps % self.factor_update_steps != 0:
            return
        name, layer = self._layers[module]
        if isinstance(grad_output, torch.Tensor):
            grad_output = (grad_output,)
        self._mini_steps_g[name] += 1
        in_hook = (
            self._update_factors_in_hook
            and self._mini_steps_g[name] % self._accumulation_steps == 0
        )
        if in_hook and self._accumulation_steps == 1 and isinstance(grad_output[0], torch.Tensor):
            decay = self.factor_decay
            group = self._assignment.factor_group(name, 'G')
            go = grad_output

            def work() -> None:
                with tracing.phase('factor_g'):
                    layer.save_and_update_g(go, alpha=decay)
                layer.reduce_g_factor(group)
            self._on_factor_stream(grad_output[0], work, 'G',
                                   last=self._layer_index[module] == 0)
            return
        self._join_factor_streams()
        with tracing.phase('factor_g'):
            if in_hook and self._accumulation_steps == 1:
                layer.save_and_update_g(grad_output, alpha=self.factor_decay)
            else:
                layer.save_layer_grad_output(grad_output)
                if in_hook:
                    layer.update_g_factor(alpha=self.factor_decay)
        if in_hook:
            layer.reduce_g_factor(self._assignment.factor_group(name, 'G'))
