"""Headline benchmark: ResNet-50 ImageNet-shaped training with distributed
K-FAC (KAISA, grad_worker_fraction=0.5) on MI355X.

Config (BASELINE.md / reference ``examples/torch_imagenet_resnet.py``):
per-GPU batch 32 at 224x224, SGD momentum 0.9, label smoothing 0.1,
K-FAC factor update every 10 steps, second-order update every 100 steps,
damping 0.001, factor decay 0.95, KL clip 0.001, hybrid-opt (gwf 0.5),
25 MB factor all-reduce buckets, eigen method with eigenvalue outer product.
Data is synthetic (random images / labels of that shape, generated on the
device), weights random-init.  fp32 by default (the reference's ImageNet
default); ``--dtype bf16`` (autocast) is also timed as the ``bf16`` field.
channels_last.

Single GPU:     python bench.py
N GPUs:         python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
                    --master-addr 127.0.0.1 --master-port P bench.py --gpus N

Prints ONE JSON line on rank 0.  ``value`` is whole-job images/s over the
K timed steps (max step time over ranks).  With ``--baseline`` (default on)
the same model is then timed without K-FAC and ``kfac_overhead_ms`` =
ms/step(K-FAC) - ms/step(SGD) is reported alongside.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

# MIOpen tuning database shipped with the repo (miopen_db/, built by
# tools/gpu_tune_miopen.sh with MIOpen find over this benchmark's
# convolutions, channels_last and NCHW): with cudnn.benchmark off, MIOpen's
# immediate mode picks the recorded fastest solution for every conv instead
# of re-running a noisy find in each process.  Must be set before MIOpen
# initialises; an explicit MIOPEN_USER_DB_PATH wins.
# Hardware queues per process: HIP's default of 4.  The eigensolver refresh
# runs its size buckets on independent streams, one per hardware queue
# (ops/linalg.py); with the native chains 4 queues beat 8 on every paired
# run (refresh step 257 / 270 / 285 ms vs 325 / 330 / 325 ms, alternating
# runs on one box: profiles/refresh_hwq_r3.txt).  Must be set before the HIP
# runtime initialises; an explicit value wins.
os.environ.setdefault('GPU_MAX_HW_QUEUES', '4')
_MIOPEN_DB = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'miopen_db')
if os.path.isdir(_MIOPEN_DB):
    os.environ.setdefault('MIOPEN_USER_DB_PATH', _MIOPEN_DB)

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd import tracing  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import step_stream  # noqa: E402
from distributed_kfac_pytorch_amd.models.resnet import get_model  # noqa: E402
from distributed_kfac_pytorch_amd.ops.cast import enable_fused_weight_cast  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import use_gemm_conv1x1  # noqa: E402
from distributed_kfac_pytorch_amd.ops.conv import use_implicit_gemm_conv  # noqa: E402

# The reference publishes no number.  Measured on MI355X: the
# upstream kfac_pytorch package, same config and harness (shipped MIOpen
# db, foreach SGD, zero_grad(set_to_none=True)), 1 GPU (it cannot run
# channels_last weights, so NCHW): 753.96 img/s
# (profiles/bench_reference_impl_mi355x_1gpu_r1c.json; 728.91 and 729.89
# under the earlier harness settings).  For N GPUs the comparison point is
# the reference's linear-scaling upper bound N * 753.96.
# bf16 (autocast) row; the fp32 row (the reference's ImageNet default, no
# --fp16, examples/torch_imagenet_resnet.py:73-76) measured the same way with
# --dtype fp32 in round 3: 692.57 img/s, 46.204 ms/step, SGD 17.711 ms/step
# (profiles/bench_reference_impl_mi355x_1gpu_fp32_r3.json).
REFERENCE_IMG_S_PER_GPU = {'bf16': 753.96, 'fp32': 692.57}
# the reference's K-FAC-only cost on the same box and harness: ms/step with
# K-FAC minus its own SGD step (bf16: 42.44 - 10.93; fp32: 46.204 - 17.711)
REFERENCE_KFAC_OVERHEAD_MS = {'bf16': 31.51, 'fp32': 28.49}



def parse_args() -> argparse.Namespace:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=100)
    p.add_argument('--warmup', type=int, default=10)
    p.add_argument('--model', default='resnet50')
    p.add_argument('--batch-size', type=int, default=32, help='per GPU')
    p.add_argument('--image-size', type=int, default=224)
    p.add_argument('--kfac-factor-update-steps', type=int, default=10)
    p.add_argument('--kfac-inv-update-steps', type=int, default=100)
    p.add_argument('--kfac-damping', type=float, default=0.001)
    p.add_argument('--kfac-factor-decay', type=float, default=0.95)
    p.add_argument('--kfac-kl-clip', type=float, default=0.001)
    p.add_argument('--kfac-grad-worker-fraction', type=float, default=0.5)
    p.add_argument('--kfac-inv-method', action='store_true',
                   help='use the damped-inverse method instead of eigen')
    p.add_argument('--no-kfac', action='store_true')
    p.add_argument('--baseline', type=int, default=1,
                   help='also time plain SGD and report the K-FAC overhead')
    p.add_argument('--no-channels-last', action='store_true')
    p.add_argument('--dtype', default='fp32', choices=['fp32', 'bf16'],
                   help='model compute dtype of the headline run: fp32 (the reference '
                        'ImageNet default, examples/torch_imagenet_resnet.py:73-76 --fp16 '
                        'off) or bf16 autocast')
    p.add_argument('--secondary-exact-fp32', type=int, default=1,
                   help='with an fp32 headline, also time the same K-FAC config with '
                        'exact-fp32 model convolutions (1x1 on hipBLASLt fp32, 3x3 on '
                        "MIOpen fp32: KFAC_CONV1X1_MATH=fp32, --conv-kxk miopen) and report "
                        'it as the exact_fp32 field')
    p.add_argument('--fp32', action='store_true', help='alias of --dtype fp32')
    p.add_argument('--bf16', action='store_true', help='alias of --dtype bf16')
    p.add_argument('--secondary-bf16', type=int, default=1,
                   help='with an fp32 headline, also time the same K-FAC config '
                        'under bf16 autocast and report it as bf16_* fields')
    p.add_argument('--phase-timing', action='store_true')
    p.add_argument('--grad-set-to-none', type=int, default=0,
                   help='zero_grad(set_to_none=...): 1 lets autograd hand its gradient '
                        'buffers to .grad (no accumulate kernels)')
    p.add_argument('--graphs', type=int, default=1,
                   help='1: replay each step kind from a captured HIP graph '
                        '(distributed_kfac_pytorch_amd.graphs.GraphedTrainStep; '
                        'single-rank jobs only, second-order update steps stay '
                        'eager); 0: every step eager')
    p.add_argument('--sgd-impl', default='fused', choices=['fused', 'foreach'],
                   help='torch.optim.SGD implementation (same math)')
    p.add_argument('--fused-weight-cast', type=int, default=1,
                   help='1: autocast weight casts by fused multi-tensor launches '
                        '(ops/cast.py; same values), 0: autocast per-weight casts')
    p.add_argument('--cudnn-benchmark', type=int, default=0,
                   help='1: MIOpen find in every process (noisy); 0: immediate mode '
                        'with the shipped tuning db (miopen_db/)')
    p.add_argument('--cudnn-deterministic', type=int, default=0,
                   help='1: MIOpen restricted to deterministic solvers (the fp32 step '
                        'becomes bit-reproducible: its strided 3x3 input gradients are '
                        'otherwise nondeterministic, tools/determinism_probe.py --fp32)')
    p.add_argument('--dump-steps', default='',
                   help='write every timed step (kind, GPU ms, host issue ms) of the '
                        'K-FAC run to this JSON file (rank 0)')
    p.add_argument('--profile-mark', action='store_true',
                   help='bracket the timed steps with marker kernels (rocprof windows)')
    p.add_argument('--conv1x1', default='gemm', choices=['miopen', 'gemm'],
                   help='1x1 convolutions: one GEMM on the NHWC activation matrix with a '
                        'slab-reduced weight gradient (ops/conv.py GemmConv1x1; same '
                        'values; default: fp32 1585.9 vs 1508.6 img/s with MIOpen, SGD '
                        'step 15.60 vs 16.67 ms, same box, profiles/r4_final/), or MIOpen')
    p.add_argument('--conv-kxk', default='gemm', choices=['miopen', 'gemm'],
                   help="3x3 convolutions: fp32 forward and stride-1 input gradient on the "
                        'native implicit-GEMM kernel (ops/conv.py ImplicitGemmConv2d), or MIOpen')
    p.add_argument('--lr', type=float, default=0.0125)
    p.add_argument('--data-pool', type=int, default=8,
                   help='distinct synthetic batches cycled through the input buffer')
    p.add_argument('--impl', default='native', choices=['native', 'reference'],
                   help='reference = time the upstream kfac_pytorch package '
                        'found on $KFAC_REFERENCE_PATH (same config) to '
                        'establish the MI355X baseline')
    p.add_argument('--backend', default='nccl',
                   help='torch.distributed backend (nccl = RCCL)')
    p.add_argument('--ddp', type=int, default=0,
                   help='1: wrap the model in DistributedDataParallel even at world 1 '
                        '(launch under torchrun: exercises RCCL init, the DDP reducer and '
                        'its capture inside the step graphs on a 1-GPU box)')
    p.add_argument('--same-device', action='store_true',
                   help='put every rank on cuda:0 (multi-rank rehearsal on a '
                        '1-GPU box; use with --backend gloo)')
    return p.parse_args()


def setup(args: argparse.Namespace) -> tuple[int, int, torch.device]:
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = 0 if args.same_device else int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    torch.backends.cudnn.deterministic = bool(args.cudnn_deterministic)
    if world > 1 or args.ddp:
        if args.graphs and (world == 1 or os.environ.get('KFAC_STEP_GRAPHS_MULTI') == '1'):
            # captured RCCL collectives: the watchdog must not poll (and
            # abort on) events recorded inside a capture
            os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '0')
        # a rank that fails leaves the others waiting in a collective: give
        # up after 5 minutes instead of the 10-minute default
        import datetime
        timeout = datetime.timedelta(seconds=300)
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev, timeout=timeout)
        else:
            dist.init_process_group(args.backend, timeout=timeout)
    return rank, world, dev


def barrier_sync(world: int) -> None:
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def _profile_marker(dev: torch.device):  # type: ignore[no-untyped-def]
    """Launch a tiny native ``identity_kernel`` at both ends of the timed
    region so ``tools/trace_summary.py --window identity_kernel`` can cut
    the steady-state steps out of a rocprofv3 kernel trace."""
    from distributed_kfac_pytorch_amd.ops import _native
    buf = torch.empty(1, 1, device=dev)
    ext = _native.native()
    assert ext is not None, _native.load_error()

    def mark() -> None:
        ext.fill_identity(buf)

    return mark


def run(args: argparse.Namespace, use_kfac: bool, rank: int, world: int,
        dev: torch.device, amp: bool) -> dict:
    torch.manual_seed(1234 + rank)
    model = get_model(args.model).to(dev)
    if args.conv1x1 == 'gemm' and args.impl == 'native':
        use_gemm_conv1x1(model)
    if args.conv_kxk == 'gemm' and args.impl == 'native':
        use_implicit_gemm_conv(model)
    cl = not args.no_channels_last
    if cl:
        model = model.to(memory_format=torch.channels_last)
    if args.fused_weight_cast and args.impl == 'native' and amp:
        # bf16 weight copies / fp32 weight gradients by multi-tensor launches
        # instead of autocast's per-weight casts (ops/cast.py)
        enable_fused_weight_cast(model)
    use_graphs = bool(args.graphs) and args.impl == 'native' and (
        world == 1 or os.environ.get('KFAC_STEP_GRAPHS_MULTI', '0') == '1')
    if world > 1 or args.ddp:
        # under graphs DDP is built on the stream the steps run and are
        # captured on (its reducer holds the AccumulateGrad nodes)
        ctx = torch.cuda.stream(step_stream(dev)) if use_graphs else contextlib.nullcontext()
        with ctx:
            model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[dev.index], gradient_as_bucket_view=True,
            )
    lr = args.lr * world
    # fused: one-pass SGD kernels (weight decay + momentum + update per
    # element); foreach: PyTorch's multi-pass multi-tensor SGD
    kw = {'fused': True} if args.sgd_impl == 'fused' else {'foreach': True}
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9,
                          weight_decay=5e-5, **kw)
    precond = None
    impl = kfac
    if use_kfac and args.impl == 'reference':
        sys.path.insert(0, os.environ['KFAC_REFERENCE_PATH'])
        import kfac as ref_kfac  # upstream package, same constructor API
        impl = ref_kfac.preconditioner
    if use_kfac:
        precond = impl.KFACPreconditioner(
            model,
            factor_update_steps=args.kfac_factor_update_steps,
            inv_update_steps=args.kfac_inv_update_steps,
            damping=args.kfac_damping,
            factor_decay=args.kfac_factor_decay,
            kl_clip=args.kfac_kl_clip,
            lr=lambda step: opt.param_groups[0]['lr'],
            accumulation_steps=1,
            allreduce_bucket_cap_mb=25,
            colocate_factors=True,
            compute_method='inverse' if args.kfac_inv_method else 'eigen',
            grad_worker_fraction=args.kfac_grad_worker_fraction,
        )
    # a pool of distinct synthetic batches, cycled through one static input
    # buffer (graph replays read it): the K-FAC factors see batch-to-batch
    # variation as with real data, so eigenbasis warm starts are not
    # flattered by a constant batch
    fmt = torch.channels_last if cl else torch.contiguous_format
    pool_x = [torch.randn(args.batch_size, 3, args.image_size, args.image_size,
                          device=dev).contiguous(memory_format=fmt)
              for _ in range(max(1, args.data_pool))]
    pool_y = [torch.randint(0, 1000, (args.batch_size,), device=dev)
              for _ in range(max(1, args.data_pool))]
    x = torch.empty_like(pool_x[0])
    y = torch.empty_like(pool_y[0])
    counter = [0]

    def next_batch() -> None:
        i = counter[0] % len(pool_x)
        counter[0] += 1
        x.copy_(pool_x[i])
        y.copy_(pool_y[i])
    crit = torch.nn.CrossEntropyLoss(label_smoothing=0.1)


    def forward_backward() -> torch.Tensor:
        # no autocast weight cache: it cannot be replayed from a graph
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=amp,
                            cache_enabled=not use_graphs):
            loss = crit(model(x), y)
        loss.backward()
        return loss

    runner = None
    if use_graphs:
        # bf16: every 1x1 conv as GEMMs inside the graphs (the tuned MIOpen
        # bf16 backward-weights solvers read outside it: ops/conv.py)
        runner = GraphedTrainStep(forward_backward, opt, precond, model=model,
                                  conv_mode='gemm' if amp else None)

    def step() -> None:
        next_batch()
        if runner is not None:
            runner()
            return
        opt.zero_grad(set_to_none=bool(args.grad_set_to_none))
        forward_backward()
        if precond is not None:
            precond.step()
        opt.step()

    def kind() -> str:
        if precond is None:
            return 'plain'
        st = precond.steps
        if st % precond.inv_update_steps == 0:
            return 'inverse'
        if st % precond.factor_update_steps == 0:
            return 'factor'
        return 'plain'

    for _ in range(args.warmup):
        step()
    # Align the timed window to the K-FAC schedule: it starts ON a
    # second-order update step, so every window (whatever --steps is)
    # contains at least one eigendecomposition/inversion refresh.  The
    # alignment steps are untimed warmup.
    align = 0
    if precond is not None:
        while precond.steps % precond.inv_update_steps != 0:
            step()
            align += 1
    timer = None
    if args.phase_timing and precond is not None:
        timer = tracing.enable_phase_timing(True)
    marker = _profile_marker(dev) if args.profile_mark else None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    kinds: list[str] = []
    barrier_sync(world)
    if marker is not None:
        marker()
    t0 = time.perf_counter()
    nan_probe = os.environ.get('KFAC_BENCH_NANSTEP') == '1'  # diagnostics only
    host_ms: list[float] = []
    for i in range(args.steps):
        kinds.append(kind())
        ev[i].record()
        h0 = time.perf_counter()
        step()
        # host time to issue the step (no sync): equal to the GPU time when
        # the step is host-bound
        host_ms.append((time.perf_counter() - h0) * 1e3)
        if nan_probe:
            bad = [n for n, p_ in model.named_parameters() if not torch.isfinite(p_).all()]
            gbad = [n for n, p_ in model.named_parameters()
                    if p_.grad is not None and not torch.isfinite(p_.grad).all()]
            if bad or gbad:
                print(f'[nan] step {i} kind {kinds[-1]}: {len(bad)} params, {len(gbad)} grads '
                      f'non-finite, e.g. {(bad or gbad)[:3]}', file=sys.stderr, flush=True)
                nan_probe = False
    ev[args.steps].record()
    if marker is not None:
        marker()
    barrier_sync(world)
    elapsed = time.perf_counter() - t0
    # per-step GPU-timeline intervals (no per-step host sync)
    per_step = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    by_kind = {}
    for k in ('plain', 'factor', 'inverse'):
        v = [t for t, kk in zip(per_step, kinds) if kk == k]
        by_kind[k] = (sum(v) / len(v)) if v else 0.0
    by_kind_local = dict(by_kind)
    t = torch.tensor([elapsed, by_kind['plain'], by_kind['factor'], by_kind['inverse']],
                     device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0].item())
    by_kind = {'plain': float(t[1]), 'factor': float(t[2]), 'inverse': float(t[3])}
    host_by_kind = {}
    for k in ('plain', 'factor', 'inverse'):
        v = sorted(t for t, kk in zip(host_ms, kinds) if kk == k)
        if v:
            host_by_kind[k] = round(v[len(v) // 2], 3)  # median
    out = {'seconds': elapsed, 'ms_per_step': elapsed / args.steps * 1e3,
           'host_issue_ms': host_by_kind,
           'kind_ms': {k: round(v, 3) for k, v in by_kind.items() if v > 0.0},
           'kind_counts': {k: kinds.count(k) for k in ('plain', 'factor', 'inverse')},
           'inverse_ms_each': [round(t, 1) for t, kk in zip(per_step, kinds) if kk == 'inverse'],
           'align_steps': align}
    if args.dump_steps and rank == 0:
        # one JSON line per timed run (K-FAC, SGD baseline, secondaries)
        with open(args.dump_steps, 'a') as f:
            f.write(json.dumps({'kfac': use_kfac, 'amp': amp, 'conv_kxk': args.conv_kxk,
                                'kinds': kinds, 'gpu_ms': [round(t, 3) for t in per_step],
                                'host_ms': [round(t, 3) for t in host_ms]}) + '\n')
    if precond is not None:
        # period-averaged step time at the reference cadence: one refresh,
        # (inv/factor - 1) factor-update steps and the rest plain steps per
        # inv_update_steps period, each at its in-window measured time
        inv_p, f_p = precond.inv_update_steps, precond.factor_update_steps
        n_factor = len([s for s in range(1, inv_p) if s % f_p == 0])
        n_plain = inv_p - 1 - n_factor
        tf = by_kind['factor'] or by_kind['plain']
        out['period_ms_per_step'] = (
            by_kind['inverse'] + n_factor * tf + n_plain * by_kind['plain']
        ) / inv_p
        out['refresh_ms'] = by_kind['inverse'] - by_kind['plain']
    if timer is not None:
        out['phase_ms_per_step'] = {
            k: v / args.steps for k, v in timer.summary().items()
        }
        out['phase_counts'] = timer.counts()
        tracing.enable_phase_timing(False)
    if runner is not None:
        out['step_graphs'] = {'replays': runner.replays, 'captures': runner.captures,
                              'eager_steps': runner.eager_steps}
        # the capture-time check per captured kind: the largest eager-vs-
        # eager relative difference over parameters / gradients (noise_max:
        # 0 for a bitwise-deterministic step) and the worst replay distance
        rep = getattr(runner, 'verify_report', None) or {}
        if rep:
            out['step_graphs']['verify'] = {
                k: {'noise_max': v.get('noise_max'), 'worst': v.get('worst'),
                    'worst_pair': v.get('worst_pair'), 'strict': v.get('strict'),
                    'ok': v.get('ok')}
                for k, v in rep.items()}
    if precond is not None and args.impl == 'native':
        out['kfac_layers'] = len(precond._layers)
        out['kfac_steps_end'] = precond.steps
        g = getattr(precond, '_graphs', None)
        if g is not None:
            out['graph_replays'] = g.replays
            out['graph_captures'] = g.captures
        mem = precond.memory_usage()
        out['kfac_memory_mb'] = round(mem['total'] / 1e6, 1)
    # numerical health of the timed run (one read-back, after the timing),
    # over every rank
    fin = torch.stack([torch.isfinite(p_).all() for p_ in model.parameters()]).all()
    fin = fin.to(torch.int32).reshape(1)
    if world > 1:
        dist.all_reduce(fin, op=dist.ReduceOp.MIN)
    out['params_finite'] = bool(fin.item())
    if precond is not None and world > 1:
        # per-rank refresh cost: KAISA places each factor's decomposition on
        # one rank, so the slowest rank sets the refresh step
        mine = torch.tensor([by_kind_local.get('inverse', 0.0)], device=dev, dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        out['refresh_ms_per_rank'] = [round(float(t.item()), 1) for t in allr]
    del model, opt, precond
    torch.cuda.empty_cache()
    return out


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return int(s.getsockname()[1])


def launcher_argv(argv: list[str], gpus: int, port: int) -> list[str]:
    """torchrun command that starts ``gpus`` ranks of this script with the
    same arguments: one process per GPU on this node, rendezvous on
    127.0.0.1 (reference launcher: ``scripts/run_imagenet.sh:54-60``)."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
            f'--nproc-per-node={gpus}', '--master-addr=127.0.0.1',
            f'--master-port={port}', '--max-restarts=0',
            os.path.abspath(__file__)] + list(argv)


def check_world(world: int, gpus: int) -> None:
    """The job must have exactly ``--gpus`` ranks: a mismatch would time a
    different configuration than the one the JSON line names."""
    if world != gpus:
        raise SystemExit(f'[bench] --gpus {gpus} but the job has {world} rank(s) '
                         f'(WORLD_SIZE={os.environ.get("WORLD_SIZE")}); launch N ranks with '
                         'torchrun or run `python bench.py --gpus N` without WORLD_SIZE set')


def main() -> None:
    args = parse_args()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # `python bench.py --gpus N`: start the N ranks as a fresh child
        # process (nothing in this process has touched the GPU), relay its
        # output (rank 0 prints the JSON line) and exit with its status
        import subprocess
        cmd = launcher_argv(sys.argv[1:], args.gpus, _free_port())
        print('[bench] launching: ' + ' '.join(cmd), file=sys.stderr, flush=True)
        sys.exit(subprocess.call(cmd))
    if args.bf16:
        args.dtype = 'bf16'
    if args.fp32:
        args.dtype = 'fp32'
    amp = args.dtype == 'bf16'
    check_world(int(os.environ.get('WORLD_SIZE', '1')), args.gpus)
    rank, world, dev = setup(args)
    res = run(args, not args.no_kfac, rank, world, dev, amp)
    base = None
    if args.baseline and not args.no_kfac:
        base = run(args, False, rank, world, dev, amp)
    sec = None
    if args.secondary_bf16 and not amp and not args.no_kfac:
        sec = run(args, True, rank, world, dev, True)
    exact = None
    if (args.secondary_exact_fp32 and not amp and not args.no_kfac and args.impl == 'native'
            and (args.conv1x1 == 'gemm' or args.conv_kxk == 'gemm')):
        # like-for-like with the reference's fp32 model math: every
        # convolution product exact fp32 (the K-FAC math stays as reported in
        # kfac_math)
        old_math = os.environ.get('KFAC_CONV1X1_MATH')
        os.environ['KFAC_CONV1X1_MATH'] = 'fp32'
        try:
            exact = run(argparse.Namespace(**{**vars(args), 'conv_kxk': 'miopen'}),
                        True, rank, world, dev, False)
        finally:
            if old_math is None:
                os.environ.pop('KFAC_CONV1X1_MATH', None)
            else:
                os.environ['KFAC_CONV1X1_MATH'] = old_math
    gb = args.batch_size * world
    window_value = gb * args.steps / res['seconds']
    # headline: period-averaged throughput (the reference baseline was timed
    # over whole 100-step periods); without K-FAC the window value
    ms = res.get('period_ms_per_step', res['ms_per_step'])
    value = gb * 1e3 / ms
    ref_per_gpu = REFERENCE_IMG_S_PER_GPU[args.dtype]
    line = {
        'impl': args.impl,
        'metric': 'images/sec (whole node), ResNet-50 ImageNet K-FAC training',
        'value': round(value, 2),
        'unit': 'images/s',
        'n_gpus': world,
        'world_size': dist.get_world_size() if dist.is_initialized() else 1,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(ms, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': round(value / (ref_per_gpu * world), 4) if ref_per_gpu else None,
        'baseline_img_s_per_gpu': ref_per_gpu,
        'dtype': args.dtype,
        'data': 'synthetic (random 224x224 images / labels, random-init '
                'weights)',
        'config': {
            'model': args.model,
            'global_batch': gb,
            'per_gpu_batch': args.batch_size,
            'seq_len': None,
            'image_size': args.image_size,
            'parallelism': f'dp{world}',
            'kfac': None if args.no_kfac else {
                'method': 'inverse' if args.kfac_inv_method else 'eigen',
                'factor_update_steps': args.kfac_factor_update_steps,
                'inv_update_steps': args.kfac_inv_update_steps,
                'grad_worker_fraction': args.kfac_grad_worker_fraction,
                'damping': args.kfac_damping,
                'kl_clip': args.kfac_kl_clip,
            },
            'channels_last': not args.no_channels_last,
            'fused_weight_cast': bool(args.fused_weight_cast) and amp,
            'sgd_impl': args.sgd_impl,
            'conv1x1': args.conv1x1,
            'conv_kxk': args.conv_kxk,
            'graphs': 'step_graphs' in res,
        },
        'timing': (
            'period-averaged: the timed window of exactly `steps` steps starts on '
            'a second-order update step; ms_per_step = (refresh step + factor '
            'steps + plain steps of one inv_update_steps period, each at its '
            'in-window time) / period' if not args.no_kfac else 'window average'
        ),
        'window_ms_per_step': round(res['ms_per_step'], 3),
        'window_images_per_sec': round(window_value, 2),
        'inverse_steps_timed': res['kind_counts']['inverse'],
        'kind_ms': res['kind_ms'],
        'kind_counts': res['kind_counts'],
    }
    if 'refresh_ms' in res:
        line['eigen_refresh_ms' if not args.kfac_inv_method else 'inverse_refresh_ms'] = round(
            res['refresh_ms'], 3)
    if base is not None:
        line['sgd_ms_per_step'] = round(base['ms_per_step'], 3)
        line['sgd_images_per_sec'] = round(gb * args.steps / base['seconds'], 2)
        line['kfac_overhead_ms'] = round(ms - base['ms_per_step'], 3)
        # the reference kfac_pytorch on the same MI355X and harness
        # 
        line['reference_kfac_overhead_ms'] = REFERENCE_KFAC_OVERHEAD_MS[args.dtype]
        line['sgd_params_finite'] = base['params_finite']
    if base is not None and 'step_graphs' in base:
        line['sgd_step_graphs'] = base['step_graphs']
    if sec is not None:
        ms2 = sec.get('period_ms_per_step', sec['ms_per_step'])
        v2 = gb * 1e3 / ms2
        line['bf16'] = {
            'value': round(v2, 2), 'ms_per_step': round(ms2, 3),
            'vs_baseline': round(v2 / (REFERENCE_IMG_S_PER_GPU['bf16'] * world), 4),
            'kind_ms': sec['kind_ms'], 'params_finite': sec['params_finite'],
            'eigen_refresh_ms': round(sec.get('refresh_ms', 0.0), 3),
            'host_issue_ms': sec['host_issue_ms'],
            # replayed from graphs (not just requested)
            'graphs': bool((sec.get('step_graphs') or {}).get('replays')),
            'step_graphs': sec.get('step_graphs'),
        }
    if exact is not None:
        ms3 = exact.get('period_ms_per_step', exact['ms_per_step'])
        v3 = gb * 1e3 / ms3
        line['exact_fp32'] = {
            'value': round(v3, 2), 'ms_per_step': round(ms3, 3),
            'vs_baseline': round(v3 / (REFERENCE_IMG_S_PER_GPU['fp32'] * world), 4),
            'kind_ms': exact['kind_ms'], 'params_finite': exact['params_finite'],
            'model_math': 'fp32 (conv1x1 hipBLASLt fp32, conv3x3 / stem MIOpen fp32)',
            'graphs': bool((exact.get('step_graphs') or {}).get('replays')),
        }
    if not args.no_kfac and args.impl == 'native':
        from distributed_kfac_pytorch_amd.ops import factors as fops
        from distributed_kfac_pytorch_amd.ops import precondition as pops
        # precision of the K-FAC math on fp32 operands: bf16x3 = three-term
        # bf16 split on MFMA (~1e-5 relative; csrc/syrk.hip, csrc/gemm3s.hip),
        # fp32 = exact fp32 products
        line['kfac_math'] = {
            'factor_syrk': 'fp32' if fops.fp32_exact() else 'bf16x3',
            'precondition': 'bf16x3' if pops.grouped_gemm_enabled() else 'fp32',
            'eigensolver': 'fp32',
        }
    if args.conv1x1 == 'gemm':
        # fp32 model math outside MIOpen: the 1x1 convolutions' forward and
        # input-gradient GEMMs (ops/conv.py conv1x1_math; ~5e-6 relative,
        # TF32 -- the reference's fp32 convolution default on NVIDIA Ampere --
        # is ~1e-3); the 3x3 convolutions and the stem's weight gradient on
        # the native implicit GEMM, the stem's forward MIOpen fp32
        from distributed_kfac_pytorch_amd.ops.conv import _conv_deterministic
        from distributed_kfac_pytorch_amd.ops.conv import conv1x1_math
        from distributed_kfac_pytorch_amd.ops.conv import conv_kxk_math
        kxk = conv_kxk_math() if args.conv_kxk == 'gemm' else 'fp32'
        det = args.conv_kxk == 'gemm' and _conv_deterministic()
        line['model_math'] = {
            'conv1x1_fwd_dgrad': conv1x1_math() if args.dtype == 'fp32' else args.dtype,
            'conv1x1_wgrad': (conv1x1_math() if args.dtype == 'fp32' else args.dtype) +
                             ' from 256x128 weights up, fp32 below',
            'conv3x3_fwd_dgrad_stride1_wgrad_ge128ch': kxk if args.dtype == 'fp32' else args.dtype,
            # KFAC_CONV_DETERMINISTIC: strided input gradients as dy . W
            # (gemm3) + fixed-order col2im, 64-channel / stem weight
            # gradients native; the stem forward stays MIOpen fp32
            'conv3x3_strided_dgrad_64ch_wgrad_stem': (
                f'{kxk} (native, deterministic); stem forward fp32 (MIOpen)' if det
                else 'fp32 (MIOpen)') if args.dtype == 'fp32' else args.dtype}
    line['host_issue_ms'] = res['host_issue_ms']
    hi = res['host_issue_ms']
    if not args.no_kfac and all(k in hi for k in ('plain', 'inverse')):
        # host time to issue one inv_update_steps period at the same cadence
        # as ms_per_step: below the GPU's period the run is not host-bound,
        # whatever a single eager step's issue time (it hides behind the
        # replays queued before it).  Meaningful for short windows: in a
        # long one the host fills the hardware queue and every issue time
        # includes the wait for a free slot
        inv_p, f_p = args.kfac_inv_update_steps, args.kfac_factor_update_steps
        n_factor = len([s_ for s_ in range(1, inv_p) if s_ % f_p == 0])
        line['period_issue_ms'] = {
            'host': round(hi['inverse'] + n_factor * hi.get('factor', hi['plain'])
                          + (inv_p - 1 - n_factor) * hi['plain'], 1),
            'gpu': round(ms * inv_p, 1)}
    if base is not None:
        line['sgd_host_issue_ms'] = base['host_issue_ms']
    for k in ('phase_ms_per_step', 'phase_counts', 'kfac_layers', 'step_graphs',
              'kfac_memory_mb', 'kfac_steps_end', 'align_steps', 'inverse_ms_each',
              'refresh_ms_per_rank', 'params_finite'):
        if k in res:
            line[k] = res[k]
    # runtime settings that serialise launches or change queueing: a box
    # with any of these set times a different program (a replayed graph
    # then blocks the host for its whole duration)
    rt = {k: v for k, v in os.environ.items()
          if k in ('HIP_LAUNCH_BLOCKING', 'AMD_SERIALIZE_KERNEL', 'AMD_SERIALIZE_COPY',
                   'GPU_MAX_HW_QUEUES', 'HIP_FORCE_DEV_KERNARG', 'DEBUG_HIP_GRAPH_PACKET_CAPTURE',
                   'HSA_ENABLE_SDMA', 'AMD_LOG_LEVEL', 'CUDA_LAUNCH_BLOCKING')}
    if rt:
        line['runtime_env'] = rt
    line['cudnn_deterministic'] = bool(args.cudnn_deterministic)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
