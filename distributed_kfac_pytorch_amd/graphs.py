"""Whole training-step HIP graphs (``GraphedTrainStep``).

A ResNet-50 step at batch 32 issues ~1,400 kernels (plus ~160 K-FAC factor
launches on factor-update steps); eager PyTorch launches them one by one from
Python, so the step is launch bound: on MI355X the plain SGD step takes
11.9 ms eagerly and 8.5 ms replayed from one captured HIP graph
(profiles/graph_step_probe_sgd.jsonl).  The reference has no equivalent (it
runs every step eagerly, with two host syncs per layer in the KL clip).

``GraphedTrainStep`` runs ``zero_grad -> forward/backward -> K-FAC step ->
optimizer step`` and captures one graph per K-FAC step *kind*:

* ``plain``: precondition + KL clip + gradient write (factors unchanged);
* ``factor``: additionally the factor SYRK/EMA launches of the forward and
  backward hooks (``steps % factor_update_steps == 0``);
* ``inverse`` steps (``steps % inv_update_steps == 0``) always run eagerly:
  the refresh runs on its own lanes and host threads (ops.linalg) and its
  finiteness check reads one flag back to the host.

Graphs are captured once ``warmup`` eager steps have run and (with K-FAC)
a second-order update step has run eagerly -- that step exercises every code
path of both kinds -- so every buffer a step touches already exists at a
fixed address: K-FAC factors, eigen bases and preconditioned-gradient
buffers are persistent.  Parameter gradients are produced inside each graph
(``zero_grad(set_to_none=True)`` before its capture), so they too sit at
fixed addresses; the descriptor tables that the grouped K-FAC kernels build
from those addresses during the capture are uploaded from pinned host
buffers the table caches keep alive (``ops.precondition._TableCache``).
Eager steps in between (second-order updates) keep the gradients allocated
(``zero_grad(set_to_none=False)``).  By default only ``plain`` steps are
replayed (``kinds``): an eager factor-update step overlaps its SYRKs with
backward on the factor side stream, which a replayed graph does not.  The
captured kinds are captured together (the other kind with the step counter
temporarily set to its next occurrence), so no capture lands inside a timed
run later.  Replays advance the host-side
K-FAC state (``steps``) exactly as an eager step would.  Values baked into a
graph -- K-FAC hyperparameters, the optimizer's learning rates -- form a
signature; when it changes the affected graphs are dropped and re-captured.

Correctness: a captured graph may only read memory that its private pool
or a live tensor owns.  MIOpen's backward-data of strided 1x1 convolutions
did not (it read free global-pool blocks, so replays broke as soon as other
eager work -- an eval pass, a second model, the refresh -- reused them), nor
do the tuned database's bf16 backward-weights solvers of some stride-1 1x1
shapes (profiles/graph_oop_r4.md).  The runner therefore switches the
model's strided 1x1 convolutions to the graph-safe
``ops.conv.StridedConv1x1`` (``conv_mode='strided'``, fp32) or every 1x1
convolution to hipBLASLt GEMMs (``conv_mode='gemm'``, required under bf16
autocast), and ``tools/graph_oop_audit.py`` / ``graph_oop_bisect.py`` check
any new model the same way (they poison the free global pool between
replays).  Every step -- eager or replayed -- runs on one persistent stream
(``step_stream()``).

Two safety nets guard every capture (round 5):

* autocast detection: the warmup eager steps record, from a forward
  pre-hook on the convolutions, whether they run under 16-bit autocast; if
  so every 1x1 convolution is switched to the GEMM form before anything is
  captured (``conv_mode`` is only a default);
* a capture-time self-check (``verify``, ``KFAC_GRAPH_VERIFY``): from one
  saved state the step runs eagerly twice and is replayed three times -- the
  second replay after an eager step of the other kind, the third straight
  after it -- and every parameter and gradient must agree per tensor within
  10x the eager-vs-eager noise (capped at 25 %, floored at twice the step's
  largest eager noise: ``verify_tolerance``); otherwise the graphs are
  dropped and the runner stays eager.

Under the bench's tuned MIOpen database (``miopen_db/``) bf16 replays are
sound: every convolution captured alone replays like its eager twin
(profiles/r5/conv_replay/), the interleaved twin test passes in a fresh
process (``tests/test_graphs_refresh_gpu.py``), and the round-4 "16.5 %
clean-replay spread" is the chaotic amplification of MIOpen's atomic
backward solvers (two EAGER runs from one state differ by 5-8 % in raw
gradients under that database: profiles/r5/tuned_db_bisect/).  The one
unsafe configuration found is ``torch.backends.cudnn.deterministic`` with
that database: MIOpen then falls back to naive direct kernels and to the CK
grouped backward-data solver, whose replays accumulate into memory the
graph never re-zeroes (a lone 3x3 conv's second replay returns twice the
first, profiles/r5/conv_replay/probe_det_tuned.jsonl, solver names in
profiles/r5/miopen_det/).  The capture-time check does not catch it (its
replays from a restored state agree with the eager step; the training
replays after them go non-finite while an eager twin stays finite:
profiles/r5/unsafe_det_bisect.log), so 16-bit autocast steps under
``cudnn.deterministic`` are never captured (``_capturable``).

Multi-rank jobs run every step eagerly by default (the K-FAC precondition
phase is still replayed from ``StepGraphs``).  The K-FAC collectives
themselves no longer block capture (``AsyncTensor`` has no host callbacks:
``Work.wait()`` only orders the current stream after RCCL's), but the DDP
gradient all-reduce does: DDP's C++ reducer launches its bucket all-reduces
from autograd hooks, rebuilds its buckets during the first iterations, and
ProcessGroupNCCL's watchdog polls each collective's HIP event from its own
thread.  Capturing that needs DDP built under the step stream (``step_stream()``),
the bucket rebuild and DDP's runtime-statistics iterations finished before
capture (``warmup`` >= 11 for a DDP model) and asynchronous error handling
off (``TORCH_NCCL_ASYNC_ERROR_HANDLING=0``).  That path is exercised at
world size 1 over RCCL (``bench.py --ddp 1`` under torchrun:
profiles/bench_r4_ddp_world1_graphs.json, 107 replays, finite); multi-GPU
capture has not been run.  ``KFAC_STEP_GRAPHS_MULTI=1`` opts a multi-rank
job in; a capture that raises falls back to eager steps on a fresh stream.
"""
from __future__ import annotations

import contextlib
import gc
import logging
import os
from collections import defaultdict
from typing import Any
from typing import Callable
from typing import Iterator

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd import tracing
from distributed_kfac_pytorch_amd.ops import _native

logger = logging.getLogger(__name__)



@contextlib.contextmanager
def _no_gc() -> Iterator[None]:
    """Collect now, then keep the cyclic GC off for the block."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()

def drain_collectives() -> None:
    """Finish every collective in flight and let each process group's RCCL
    watchdog retire its work list before a capture starts.

    ProcessGroupNCCL's watchdog thread polls the HIP end event of every
    eager collective until it has completed.  A query that lands while this
    thread captures in ``global`` mode is an illegal call under capture: it
    invalidates the capture and the watchdog dies on the error, which aborts
    the process (SIGABRT: the round-5 driver failure of
    ``tests/test_rccl_gpu.py``, timing dependent because the watchdog polls
    every ~100 ms).  Captures here use ``thread_local`` mode, which leaves
    other threads' calls alone; draining first removes the race entirely.
    """
    if not torch.cuda.is_available():
        return
    torch.cuda.synchronize()
    if not (dist.is_available() and dist.is_initialized()):
        return
    try:
        groups = list(dist.distributed_c10d._world.pg_map.keys())
    except Exception:  # noqa: BLE001
        groups = [dist.distributed_c10d._get_default_group()]
    for pg in groups:
        try:
            pg._wait_for_pending_works()
        except Exception:  # noqa: BLE001 -- backends without a work list (gloo)
            pass


_STEP_STREAMS: dict = {}


def step_stream(device: torch.device | int | None = None) -> torch.cuda.Stream:
    """The per-device stream ``GraphedTrainStep`` runs steps and captures on
    by default.  Construct a ``DistributedDataParallel`` model under it
    (``with torch.cuda.stream(step_stream()):``) when its steps will be
    graph-captured."""
    if device is None:
        dev = torch.cuda.current_device()
    elif isinstance(device, int):
        dev = device
    else:
        dev = device.index if device.index is not None else torch.cuda.current_device()
    s = _STEP_STREAMS.get(dev)
    if s is None:
        # KFAC_STEP_STREAM_PRIORITY (default 0; -1 = high): a high-priority
        # step stream lets the forward / backward kernels dispatch ahead of
        # the factor SYRKs of the side stream (priority 0)
        prio = int(os.environ.get('KFAC_STEP_STREAM_PRIORITY', '0'))
        s = torch.cuda.Stream(device=dev, priority=prio)
        _STEP_STREAMS[dev] = s
    return s


def verify_tolerance(noise: torch.Tensor) -> torch.Tensor:
    """Per-tensor tolerance of the capture-time check from the eager-vs-eager
    relative distances ``noise`` (one entry per parameter / gradient).

    ``min(10 x n, max(2 x n, 0.25))`` of the tensor's own noise ``n`` -- a
    replay may be ten times as noisy as one eager pair, but not 25 % off when
    the eager pair agrees to within 12.5 % -- plus a floor of twice the
    step's largest eager noise (capped at 25 %) and 1e-3.  The floor: one
    eager pair under-samples the noise of a tensor fed by atomic reductions
    (MIOpen's bf16 solvers), and replays reorder those atomics more than two
    back-to-back eager steps do.  In the ImageNet CLI's bf16 batch-8 steps six
    eager steps from one state spread by up to 14 % in BatchNorm gradients,
    six replays by 10-16 % around the eager step AND around each other, yet
    single eager pairs put some of those tensors at 0 - 1e-4 and the check
    dropped sound graphs in half the runs (profiles/r5/graph_verify_probe/;
    with a floor of 1x the largest noise, one run in ~10 still failed: 12 %
    against a 6.9 % step noise, profiles/r5/pytest_gpu_final/).  The hazards the check exists for
    (memory a graph reads outside its pool, accumulation the graph never
    re-zeroes) move a gradient by O(1) or make it non-finite; a deterministic
    fp32 step keeps a floor of ~1e-3 (its eager noise is zero, so is the
    floor).  The floor is applied to every tensor, including ones the single
    eager pair reproduced bit for bit: in the ImageNet CLI's bf16 steps one
    BatchNorm gradient with zero eager-pair noise differed by 12 % between
    replay and eager while the step's largest noise was 8.9 % -- the same
    atomic noise, unsampled (a round-6 attempt to exempt zero-noise tensors
    dropped those sound graphs: profiles/r6/pytest_gpu_r6b_tolerance.log).
    A non-finite noise entry makes every tolerance NaN (the check fails)."""
    floor = torch.clamp(2.0 * noise.max(), max=0.25) if noise.numel() else noise.new_zeros(())
    return torch.minimum(10.0 * noise, torch.clamp(2.0 * noise, min=0.25)) + floor + 1e-3


def verify_ratio(d: torch.Tensor, tol: torch.Tensor, strict: bool) -> torch.Tensor:
    """Distance over tolerance per tensor (> 1 fails; non-finite distances
    are infinite).  ``strict`` (the eager step reproduced itself bit for
    bit: every noise entry zero, e.g. the fp32 ResNet-50 step with
    ``KFAC_CONV_DETERMINISTIC``): any nonzero distance fails -- a replay of a
    deterministic step must be bit-identical to the eager step."""
    inf = torch.full_like(d, float('inf'))
    if strict:
        return torch.where(d == 0, torch.zeros_like(d), inf)
    return torch.where(torch.isfinite(d), d / tol, inf)


def _graph_safe(model: torch.nn.Module | None, preconditioner: Any,
                mode: str | None = None) -> int:
    from distributed_kfac_pytorch_amd.ops.conv import StridedConv1x1
    from distributed_kfac_pytorch_amd.ops.conv import make_graph_safe

    n = make_graph_safe(model, mode) if model is not None else 0
    for module in list(getattr(preconditioner, '_layers', None) or {}):
        if type(module) in (torch.nn.Conv2d, StridedConv1x1) and module.kernel_size == (1, 1):
            n += make_graph_safe(module, mode)
    return n


class GraphedTrainStep:
    """Run (and graph-capture) a full training step.

    Args:
        forward_backward: callable that runs forward + backward on static
            input tensors and returns the loss (a tensor).  It must not call
            ``zero_grad`` / ``preconditioner.step`` / ``optimizer.step``:
            the runner does.
        optimizer: the torch optimizer.
        preconditioner: a ``BaseKFACPreconditioner`` or None (plain SGD).
        warmup: eager steps (after construction or a hyperparameter change)
            before the graphs are captured.
        enabled: force graphs on / off (default: on when CUDA is available
            and the job has a single rank).
        model: the trained module; its 1x1 convolutions are switched to the
            graph-safe formulation of ``ops.conv`` (same parameters and
            values).  Without it only K-FAC's registered layers are.
        conv_mode: ``ops.conv.make_graph_safe`` mode: ``'strided'`` (fp32
            default: strided 1x1 convolutions only) or ``'gemm'`` (every 1x1
            convolution as hipBLASLt GEMMs; REQUIRED when the step runs under
            bf16 autocast, whose tuned MIOpen backward-weights solvers read
            memory outside the graph: profiles/graph_oop_r4.md).  Default:
            ``KFAC_GRAPH_SAFE_CONV``, else ``'strided'``.
        stream: the HIP stream every step -- eager or replayed -- and every
            capture runs on (default: a private stream; the caller's stream
            is joined on entry and exit).  One stream for all of them keeps
            the autograd engine's AccumulateGrad nodes on the stream that
            produces the gradients.  A ``DistributedDataParallel`` model must
            be CONSTRUCTED under it (``with torch.cuda.stream(step.stream)``,
            or ``step_stream()`` before building the runner): DDP's reducer
            holds every parameter's AccumulateGrad node from construction
            on, and nodes bound to another stream make the captured backward
            synchronise with a stream outside the capture.
    """

    def __init__(
        self,
        forward_backward: Callable[[], torch.Tensor],
        optimizer: torch.optim.Optimizer,
        preconditioner: Any = None,
        *,
        warmup: int = 1,
        enabled: bool | None = None,
        kinds: tuple[str, ...] = ('plain',),
        model: torch.nn.Module | None = None,
        stream: torch.cuda.Stream | None = None,
        conv_mode: str | None = None,
        verify: bool | None = None,
    ) -> None:
        self.forward_backward = forward_backward
        self.model = model
        self.optimizer = optimizer
        self.preconditioner = preconditioner
        if isinstance(model, torch.nn.parallel.DistributedDataParallel):
            # DDP records runtime statistics (event timings, host syncs) in
            # its first 10 iterations: a capture must come after them
            warmup = max(warmup, 11)
        self.warmup = warmup
        if enabled is None:
            multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
            enabled = torch.cuda.is_available() and (
                not multi or os.environ.get('KFAC_STEP_GRAPHS_MULTI', '0') == '1'
            )
        self.enabled = enabled
        self.stream = stream
        if enabled and self.stream is None:
            self.stream = step_stream()
        self.conv_mode = conv_mode or os.environ.get('KFAC_GRAPH_SAFE_CONV', 'strided')
        if enabled:
            # 1x1 convolutions through the graph-safe formulations (some
            # MIOpen solvers read memory outside the graph: ops/conv.py); the
            # model's, or at least K-FAC's layers'
            _graph_safe(model, preconditioner, self.conv_mode)
        if verify is None:
            verify = os.environ.get('KFAC_GRAPH_VERIFY', '1') != '0'
        self.verify = verify
        # autocast seen by a convolution during the eager warmup steps
        self.autocast_dtype: torch.dtype | None = None
        self._probe_handles: list = []
        self.verify_report: dict[str, dict] = {}
        # Step kinds replayed from graphs.  Factor-update steps stay eager by
        # default: their SYRKs run on the factor side stream concurrently with
        # backward, and a replayed graph executes its nodes in one queue, so
        # the captured factor step was slower than the eager one (ResNet-50
        # fp32: 24.9 vs 22.6 ms, 1485 vs 1555 img/s;
        # profiles/bench_r3_fp32_fusedbn_*graphs.json).  KFAC_GRAPH_KINDS
        # overrides (e.g. "plain,factor").
        env = os.environ.get('KFAC_GRAPH_KINDS')
        if env:
            kinds = tuple(k.strip() for k in env.split(',') if k.strip())
        self.kinds = tuple(k for k in kinds if k in ('plain', 'factor'))
        if enabled and preconditioner is not None and getattr(preconditioner, '_graphs', None):
            # The whole-step graph already contains the precondition phase.
            # With the preconditioner's own precondition-phase graphs
            # (StepGraphs) also active, the replays after capture produced
            # garbage preconditioned gradients from the first replay on, while
            # with StepGraphs off the replays matched the eager twin exactly
            # (ResNet-50, bf16 and fp32:
            # profiles/graph_replay_stepgraphs_r3.txt).
            preconditioner._graphs = None
        self.graphs: dict[str, torch.cuda.CUDAGraph] = {}
        self.outputs: dict[str, torch.Tensor] = {}
        self.grads: dict[str, list] = {}
        self.seen = 0
        self.signature: tuple | None = None
        self.replays = 0
        self.captures = 0
        self.eager_steps = 0
        self._inverse_done = preconditioner is None
        self._caller: torch.cuda.Stream | None = None

    # ------------------------------------------------------------ helpers
    def kind(self) -> str:
        """The K-FAC step kind of the next step."""
        p = self.preconditioner
        if p is None:
            return 'plain'
        s = p.steps
        if s % p.inv_update_steps == 0:
            return 'inverse'
        if s % p.factor_update_steps == 0:
            return 'factor'
        return 'plain'

    def _signature(self) -> tuple:
        lrs = tuple(float(g['lr']) for g in self.optimizer.param_groups)
        p = self.preconditioner
        if p is None:
            return lrs
        kl = p.kl_clip
        return lrs + (float(p.damping), float(p.factor_decay),
                      None if kl is None else float(kl), float(p.lr),
                      int(p.factor_update_steps), int(p.inv_update_steps))

    def _params(self) -> list:
        return [q for group in self.optimizer.param_groups for q in group['params']]

    def _conv_modules(self) -> list:
        mods = list(self.model.modules()) if self.model is not None else [
            layer.module.module for _, layer in
            (getattr(self.preconditioner, '_layers', None) or {}).values()]
        return [m for m in mods if isinstance(m, torch.nn.Conv2d)]

    def _probe_autocast(self) -> None:
        """Record, from a forward pre-hook on the convolutions, whether the
        step runs them under 16-bit autocast (removed again after the step)."""
        def hook(mod: torch.nn.Module, inp: Any) -> None:
            if torch.is_autocast_enabled('cuda'):
                dt = torch.get_autocast_dtype('cuda')
                if dt in (torch.bfloat16, torch.float16):
                    self.autocast_dtype = dt
        self._probe_handles = [m.register_forward_pre_hook(hook) for m in self._conv_modules()]

    def _end_probe(self) -> None:
        for h in self._probe_handles:
            h.remove()
        self._probe_handles = []
        if self.autocast_dtype is not None and self.conv_mode != 'gemm':
            # MIOpen's tuned 16-bit 1x1 backward-weights solvers read memory
            # outside a captured graph (ops/conv.py): every 1x1 convolution
            # goes through the GEMM formulation before anything is captured
            n = _graph_safe(self.model, self.preconditioner, 'gemm')
            logger.warning('step runs under %s autocast: conv_mode %r -> \'gemm\' '
                           '(%d 1x1 convolutions as GEMMs)', self.autocast_dtype,
                           self.conv_mode, n)
            self.conv_mode = 'gemm'

    def _eager(self) -> torch.Tensor:
        probe = self.enabled and not self.graphs and self.captures == 0
        if probe:
            self._probe_autocast()
        try:
            loss = self._eager_step()
        finally:
            if probe:
                self._end_probe()
        self.eager_steps += 1
        # detached: a caller holding the loss must not keep this step's
        # autograd graph (and its AccumulateGrad nodes, bound to the eager
        # stream) alive across the next capture
        return loss.detach()

    def _eager_step(self) -> torch.Tensor:
        # (Dropping the gradients here instead -- autograd's buffers handed
        # over, no accumulate kernels -- was measured in round 6: the factor
        # step's GPU time did not move, 17.39 vs 17.43 ms, and its host issue
        # rose 12.6 -> 16.5 ms (fp32) and 18.4 -> 26.7 ms (bf16) rebuilding
        # the grouped kernels' descriptor tables for the new addresses:
        # profiles/r6/eager_set_to_none/.)
        self.optimizer.zero_grad(set_to_none=False)
        loss = self.forward_backward()
        if self.preconditioner is not None:
            self.preconditioner.step()
        self.optimizer.step()
        return loss

    def _advance(self) -> None:
        """Host-side K-FAC state change of one replayed step."""
        p = self.preconditioner
        if p is not None:
            p._steps += 1
            p._mini_steps = defaultdict(int)
            p._mini_steps_g = defaultdict(int)

    def _capturable(self) -> bool:
        if self.autocast_dtype is not None and torch.backends.cudnn.deterministic:
            # 16-bit convolutions with cudnn.deterministic: MIOpen falls back
            # to its naive direct kernels and to the CK grouped backward-data
            # solver, whose captured replays accumulate into memory the graph
            # never re-zeroes (profiles/r5/conv_replay/probe_det_tuned.jsonl).
            # The capture-time check cannot be relied on here: its replays
            # from a restored state pass and the training replays after them
            # go non-finite (profiles/r5/unsafe_det_bisect.log).  Eager only.
            if self.enabled:
                logger.warning('16-bit autocast with cudnn.deterministic: step graphs '
                               'disabled (MIOpen deterministic solvers are not replay-safe)')
                self.enabled = False
            return False
        p = self.preconditioner
        if p is None:
            return True
        if p._accumulation_steps != 1:
            return False
        for _, layer in p._layers.values():
            if layer.a_factor is None or layer.g_factor is None:
                return False
        return self._inverse_done

    def _next_step_of(self, kind: str) -> int | None:
        """The next K-FAC step number (>= now) of the given kind."""
        p = self.preconditioner
        if p is None:
            return 0
        f, inv = p.factor_update_steps, p.inv_update_steps
        for s in range(p.steps, p.steps + 4 * f * inv + 2):
            if s % inv == 0:
                continue
            if (s % f == 0) == (kind == 'factor'):
                return s
        return None

    def _capture(self, kind: str) -> None:
        p = self.preconditioner
        saved = p._steps if p is not None else 0
        self._steps_before_capture = saved
        if p is not None:
            at = self._next_step_of(kind)
            if at is None:
                return
            p._steps = at
        g = torch.cuda.CUDAGraph()
        side = self.stream if self.stream is not None else torch.cuda.Stream()
        if side != torch.cuda.current_stream():
            side.wait_stream(torch.cuda.current_stream())
        # Gradients are dropped before the capture, so the captured backward
        # writes them directly (autograd hands over its buffer, no
        # zero + accumulate kernels: ~160 fewer launches and 0.8 ms per
        # ResNet-50 step) into this graph's private pool, where they stay
        # at fixed addresses for every replay.
        self.optimizer.zero_grad(set_to_none=True)
        # every eager collective retired by its watchdog before capturing
        drain_collectives()
        # no Python GC while capturing: collecting an unreachable cycle that
        # holds an old CUDAGraph would destroy that graph mid-capture, which
        # HIP forbids (hipErrorStreamCaptureUnsupported -> abort).
        # thread_local capture mode: calls from other threads (RCCL's
        # watchdog, the refresh lanes) neither invalidate this capture nor
        # fail themselves.
        with _no_gc(), torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side, capture_error_mode='thread_local'):
                loss = self.forward_backward()
                if p is not None:
                    p.step()
                self.optimizer.step()
        if side != torch.cuda.current_stream():
            torch.cuda.current_stream().wait_stream(side)
        # descriptor tables built during the capture: one eager upload now
        _native.flush_table_uploads()
        if p is not None:
            # capture ran the step's host code without executing it
            p._steps = saved
            p._mini_steps = defaultdict(int)
            p._mini_steps_g = defaultdict(int)
        self.graphs[kind] = g
        # Keep only the loss VALUE (replays rewrite its storage).  Holding the
        # captured loss itself keeps its autograd graph alive, and with it
        # every parameter's AccumulateGrad node -- created during the capture
        # and bound to the capture's side stream.  The next EAGER step (the
        # second-order refresh) then reuses those nodes: each gradient is
        # accumulated on that foreign stream while the producing stream has
        # already recycled the incoming gradient's memory, so the refresh
        # step folds garbage into the gradients / factors and the replays
        # after it diverge (profiles/graph_replay_nonfinite_r2.txt; torch
        # warns "The AccumulateGrad node's stream does not match ...").
        self.outputs[kind] = loss.detach()
        del loss
        self.grads[kind] = [q.grad for q in self._params()]
        self.captures += 1

    # ------------------------------------------------------- verification
    def _state(self, kind: str) -> list[torch.Tensor]:
        """Every tensor a step of ``kind`` reads and writes besides its
        inputs: parameters, module buffers (BN statistics), optimizer state
        and the K-FAC factors."""
        out: list[torch.Tensor] = []
        seen: set[int] = set()

        def add(t: Any) -> None:
            if isinstance(t, torch.Tensor) and t.is_cuda and id(t) not in seen:
                seen.add(id(t))
                out.append(t)
        for q in self._params():
            add(q)
        if self.model is not None:
            for b in self.model.buffers():
                add(b)
        for st in self.optimizer.state.values():
            for v in st.values():
                add(v)
        p = self.preconditioner
        if p is not None:  # the check also runs an eager factor-update step
            for _, layer in p._layers.values():
                add(layer.a_factor)
                add(layer.g_factor)
        return out

    def _verify(self, kind: str) -> bool:
        """Capture-time self-check of the ``kind`` graph.

        From one saved state (and CUDA RNG state) run the step eagerly twice
        and replay the graph three times: the second replay after an eager
        step of the other kind, the third straight after the second.  Eager vs eager is the noise floor of the
        step's nondeterministic kernels (atomics in MIOpen solvers), measured
        per tensor; every parameter (relative to its update) and every
        gradient (relative to its norm) of every replay must agree with the
        eager step, and the replays with each other, within
        ``verify_tolerance`` of that tensor's noise, and be finite.  Per tensor, because a solver
        that corrupts one layer's input gradient (MIOpen's deterministic
        bf16 backward-data under the tuned database accumulates into memory
        the graph never re-zeroes: profiles/r5/conv_replay/) hides in a
        whole-model norm behind the large layers.  A graph that depends on memory
        or library state outside the capture (the round-2..4 failures:
        free global-pool blocks, MIOpen solvers) fails it.  The state is
        restored afterwards."""
        p = self.preconditioner
        state = self._state(kind)
        with torch.no_grad():
            saved = [t.detach().clone() for t in state]
        rng = torch.cuda.get_rng_state()
        steps = p._steps if p is not None else 0
        at = self._next_step_of(kind) if p is not None else 0
        params = self._params()

        def restore() -> None:
            # factor SYRKs an eager step left running on the side stream
            # (lazy G join) finish before their outputs are overwritten
            if p is not None and hasattr(p, 'sync_factors'):
                p.sync_factors()
            with torch.no_grad():
                for t, s0 in zip(state, saved):
                    t.copy_(s0)
            torch.cuda.set_rng_state(rng)

        def snap(grads: list) -> tuple[list, list]:
            return ([q.detach().clone() for q in params],
                    [None if g is None else g.detach().clone() for g in grads])

        def eager(step_at: int | None = None) -> tuple[list, list]:
            restore()
            if p is not None:
                p._steps = at if step_at is None else step_at
            self._eager_step()
            if p is not None:
                if hasattr(p, 'sync_factors'):
                    p.sync_factors()
                p._steps = steps
                p._mini_steps = defaultdict(int)
                p._mini_steps_g = defaultdict(int)
            return snap([q.grad for q in params])

        def replay() -> tuple[list, list]:
            restore()
            self.graphs[kind].replay()
            return snap(self.grads[kind])

        p0 = [q.detach().clone() for q in params]
        e1, e2 = eager(), eager()
        r1 = replay()
        # the second replay follows an eager step of the OTHER kind -- what
        # runs between replays in training (a factor-update step between
        # plain replays): a graph that depends on state an eager step
        # rewrites (MIOpen's deterministic bf16 backward-data under the tuned
        # database: profiles/r5/) fails here, not on back-to-back replays
        other = None
        if p is not None:
            other = self._next_step_of('factor' if kind == 'plain' else 'plain')
        eager(other)
        r2 = replay()
        # ... and a third replay straight after the second, as plain steps
        # replay back to back in training: a graph whose kernels accumulate
        # into memory only an eager call re-zeroes (the deterministic
        # backward-data solver above) passes r1 and r2 and fails here
        r3 = replay()
        restore()

        idx = [i for i, g in enumerate(e1[1]) if g is not None]

        @torch.no_grad()
        def rel(xs: list, ys: list, refs: list) -> torch.Tensor:
            num = torch.stack(torch._foreach_norm(torch._foreach_sub(xs, ys))).double()
            den = torch.stack(torch._foreach_norm(refs)).double()
            inf = torch.full_like(num, float('inf'))
            return torch.where(den > 0, num / den.clamp_min(1e-300),
                               torch.where(num > 0, inf, torch.zeros_like(num)))

        def dist(a: tuple, b: tuple) -> torch.Tensor:
            # per tensor: parameters relative to the eager update, gradients
            # relative to the eager gradient
            upd = torch._foreach_sub(e1[0], p0)
            dp = rel(a[0], b[0], upd)
            ga = [a[1][i] for i in idx]
            gb = [b[1][i] for i in idx]
            dg = rel(ga, gb, [e1[1][i] for i in idx])
            return torch.cat([dp, dg])

        names = [f'param[{i}]' for i in range(len(params))] + [f'grad[{i}]' for i in idx]
        noise = dist(e2, e1)
        tol = verify_tolerance(noise)
        # KFAC_GRAPH_VERIFY_STRICT (default 1): a bit-reproducible eager
        # step demands bit-identical replays
        strict = (os.environ.get('KFAC_GRAPH_VERIFY_STRICT', '1') == '1'
                  and noise.numel() > 0 and float(noise.max()) == 0.0)
        worst_ratio, worst_at, worst, worst_pair, worst_noise = 0.0, None, 0.0, None, 0.0
        runs = {'e1': e1, 'r1': r1, 'r2': r2, 'r3': r3}
        for pa, pb in (('r1', 'e1'), ('r2', 'e1'), ('r3', 'e1'), ('r2', 'r1'), ('r3', 'r1')):
            d = dist(runs[pa], runs[pb])
            ratio = verify_ratio(d, tol, strict)
            r, i = (float(v) for v in torch.max(ratio, 0))
            if r > worst_ratio or worst_at is None:
                worst_ratio, worst_at, worst = r, names[int(i)], float(d[int(i)])
                worst_pair = f'{pa}-{pb}'
                worst_noise = float(noise[int(i)])
        finite = all(bool(torch.isfinite(t).all()) for r in (r1, r2, r3)
                     for t in list(r[0]) + [g for g in r[1] if g is not None])
        ok = finite and worst_ratio <= 1.0  # NaN compares False
        self.verify_report[kind] = {'noise_max': float(noise.max()), 'worst': worst,
                                    'worst_tensor': worst_at, 'worst_pair': worst_pair,
                                    'worst_noise': worst_noise, 'worst_over_tol': worst_ratio,
                                    'finite': finite, 'strict': strict, 'ok': ok}
        if not ok:
            logger.warning('step graph %r failed its capture-time check (%s differs by %.3g '
                           'in %s, %.3g x its tolerance; finite %s): graphs dropped, running '
                           'eagerly', kind, worst_at, worst, worst_pair, worst_ratio, finite)
        return ok

    def _drop_graphs(self) -> None:
        """Give up on graphs: run every later step eagerly, on a fresh
        stream ordered after the caller's and the old step stream's work."""
        old = self.stream
        self.enabled = False
        self.stream = torch.cuda.Stream()
        self.stream.wait_stream(self._caller or torch.cuda.current_stream())
        if old is not None:
            self.stream.wait_stream(old)
        self.graphs.clear()
        self.outputs.clear()
        self.grads.clear()
        # tables built during the failed capture serve the eager steps too;
        # upload them from the new stream (the old one may still report the
        # invalidated capture)
        with torch.cuda.stream(self.stream):
            _native.flush_table_uploads()
        gc.collect()

    def close(self) -> None:
        """Release the captured graphs (and their pools) now.

        Call before ``dist.destroy_process_group()``: a graph that captured
        RCCL collectives holds references into the communicator, and
        destroying it after the communicator (at interpreter exit, or when
        the garbage collector gets to it) touches freed state."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self.graphs.clear()
        self.outputs.clear()
        self.grads.clear()
        self.enabled = False
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    # --------------------------------------------------------------- step
    def __call__(self) -> torch.Tensor:
        caller = torch.cuda.current_stream() if torch.cuda.is_available() else None
        self._caller = caller
        if not self.enabled or self.stream is None or caller == self.stream:
            out = self._call()
            if self.stream is not None and caller is not None and caller != self.stream:
                caller.wait_stream(self.stream)  # graphs were dropped mid-call
            return out
        self.stream.wait_stream(caller)
        with torch.cuda.stream(self.stream):
            out = self._call()
        caller.wait_stream(self.stream)
        return out

    def _call(self) -> torch.Tensor:
        kind = self.kind()
        if not self.enabled or kind == 'inverse':
            loss = self._eager()
            self.seen += 1
            if kind == 'inverse':
                self._inverse_done = True
            return loss
        sig = self._signature()
        if sig != self.signature:
            if self.graphs:
                logger.info('hyperparameters changed: dropping %d step graphs', len(self.graphs))
            self.graphs.clear()
            self.outputs.clear()
            self.grads.clear()
            self.signature = sig
            self.seen = 0
        if kind not in self.graphs:
            if self.seen < self.warmup or not self._capturable():
                self.seen += 1
                return self._eager()
            kinds = self.kinds if self.preconditioner is not None else ('plain',)
            if self.preconditioner is not None and hasattr(self.preconditioner, 'sync_factors'):
                # factor SYRKs the last eager step left running (the lazy
                # join): done before the state is saved and the capture starts
                self.preconditioner.sync_factors()
            for k in kinds:
                if k not in self.graphs:
                    failed = None
                    try:
                        self._capture(k)
                    except Exception as e:  # noqa: BLE001
                        failed = repr(e)
                    if failed is None and self.verify and k in self.graphs:
                        if not self._verify(k):
                            failed = f'capture-time check failed: {self.verify_report[k]}'
                    if failed is not None:
                        # something in the step is not capturable: run eagerly.
                        # (Outside the except block: the exception's traceback
                        # holds the failed capture's loss, and with it
                        # AccumulateGrad nodes bound to the capture stream.)
                        logger.warning('step graph capture failed (%s); running eagerly', failed)
                        if self.preconditioner is not None:
                            self.preconditioner._steps = self._steps_before_capture
                        # a stream whose capture was invalidated is not reused
                        self._drop_graphs()
                        with torch.cuda.stream(self.stream):
                            return self._eager()
            if kind not in self.graphs:
                return self._eager()
        with tracing.phase(f'step(graph:{kind})'):
            self.graphs[kind].replay()
        # expose this graph's gradients as .grad (each kind has its own)
        for q, gr in zip(self._params(), self.grads[kind]):
            q.grad = gr
        self._advance()
        self.replays += 1
        return self.outputs[kind]
