"""torchrun worker of ``tests/test_rccl_gpu.py`` (not collected by pytest).

One rank per GPU over the ``nccl`` backend (RCCL on ROCm): DDP + K-FAC +
``GraphedTrainStep`` on a CIFAR ResNet-20, the DDP model built under the
step stream so its reducer's all-reduces are captured inside the step graphs
(``graphs.py``), then the same seed without DDP, eagerly.  Prints one JSON
line with what the test asserts.
"""
from __future__ import annotations

import faulthandler
import gc
import json
import os
import sys

os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '0')  # captured collectives
# a fatal signal (SIGABRT from a C++ terminate) prints every thread's Python
# stack to stderr, which the test keeps in full
faulthandler.enable(all_threads=True)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import distributed_kfac_pytorch_amd as kfac  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import GraphedTrainStep  # noqa: E402
from distributed_kfac_pytorch_amd.graphs import step_stream  # noqa: E402
from distributed_kfac_pytorch_amd.models.cifar_resnet import resnet20  # noqa: E402

STEPS = 40


def train(dev: torch.device, ddp: bool) -> dict:
    torch.manual_seed(0)
    model = resnet20().to(dev).to(memory_format=torch.channels_last)
    if ddp:
        with torch.cuda.stream(step_stream(dev)):
            model = torch.nn.parallel.DistributedDataParallel(
                model, device_ids=[dev.index], gradient_as_bucket_view=True)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    pre = kfac.KFACPreconditioner(model, factor_update_steps=2, inv_update_steps=10,
                                  damping=0.003, kl_clip=0.001,
                                  lr=lambda s: opt.param_groups[0]['lr'])
    gen = torch.Generator(device='cpu').manual_seed(1)
    pool = [(torch.randn(32, 3, 32, 32, generator=gen), torch.randint(0, 10, (32,), generator=gen))
            for _ in range(4)]
    x = torch.empty(32, 3, 32, 32, device=dev).contiguous(memory_format=torch.channels_last)
    y = torch.empty(32, dtype=torch.long, device=dev)
    crit = torch.nn.CrossEntropyLoss()

    def fb() -> torch.Tensor:
        loss = crit(model(x), y)
        loss.backward()
        return loss

    runner = None
    if ddp:
        runner = GraphedTrainStep(fb, opt, pre, model=model, kinds=('plain', 'factor'))
    losses = []
    for i in range(STEPS):
        xs, ys = pool[i % len(pool)]
        x.copy_(xs)
        y.copy_(ys)
        if runner is not None:
            loss = runner()
        else:
            opt.zero_grad(set_to_none=False)
            loss = fb()
            pre.step()
            opt.step()
        losses.append(loss.detach().clone())
    torch.cuda.synchronize()
    net = model.module if ddp else model
    replays = runner.replays if runner is not None else 0
    captures = runner.captures if runner is not None else 0
    verify = runner.verify_report if runner is not None else {}
    if runner is not None:
        # graphs holding captured RCCL work go before the communicator does
        runner.close()
    print(f'[worker] ddp={ddp} steps={STEPS} replays={replays} captures={captures}',
          flush=True)
    return {
        'losses': [float(v) for v in losses],
        'params': [p.detach().clone() for p in net.parameters()],
        'replays': replays,
        'captures': captures,
        'verify': verify,
        'finite': all(bool(torch.isfinite(p).all()) for p in net.parameters()),
    }


def main() -> None:
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    dist.init_process_group('nccl', device_id=dev)
    backend = dist.get_backend()
    a = train(dev, ddp=True)
    dist.barrier()
    b = train(dev, ddp=False)
    diff = max(float((p - q).norm() / q.norm().clamp_min(1e-12))
               for p, q in zip(a['params'], b['params']))
    out = {'backend': backend, 'world': dist.get_world_size(), 'replays': a['replays'],
           'captures': a['captures'], 'verify': a['verify'], 'finite': a['finite'],
           'param_rel_diff': diff, 'loss_ddp': a['losses'][-1], 'loss_plain': b['losses'][-1],
           'max_loss_diff': max(abs(u - v) for u, v in zip(a['losses'], b['losses']))}
    if dist.get_rank() == 0:
        print('RESULT ' + json.dumps(out), flush=True)
    dist.barrier()
    gc.collect()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print('[worker] process group destroyed', flush=True)


if __name__ == '__main__':
    main()
