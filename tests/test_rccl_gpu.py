"""K-FAC over RCCL (the ``nccl`` backend) in the GPU suite.

The rest of the suite joins ranks with gloo; this test starts a fresh
``torch.distributed.run`` child (one rank, ``--nproc-per-node 1``: RCCL
refuses two ranks on one GPU) before anything in that process touches the
GPU, and the worker (``tests/_rccl_worker.py``) trains a CIFAR ResNet-20 with
DDP + K-FAC + whole-step graphs over ``nccl`` -- DDP's reducer all-reduces
captured inside the step graphs -- and then the same seed without DDP,
eagerly.  Reference usage: ``examples/torch_imagenet_resnet.py:246-251``
(``dist.init_process_group('nccl')`` + DDP + K-FAC).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return int(s.getsockname()[1])


def test_ddp_kfac_graphs_over_rccl(cuda) -> None:
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env['PYTHONUNBUFFERED'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', f'--master-port={_port()}',
           os.path.join(ROOT, 'tests', '_rccl_worker.py')]
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith('RESULT ')]
    assert proc.returncode == 0 and lines, (proc.returncode, proc.stdout[-3000:],
                                            proc.stderr[-3000:])
    out = json.loads(lines[-1][len('RESULT '):])
    assert out['backend'] == 'nccl', out
    assert out['world'] == 1
    assert out['finite'], out
    # plain and factor-update steps replayed, each passed its capture check
    assert out['captures'] == 2 and out['replays'] >= 15, out
    assert all(r['ok'] for r in out['verify'].values()) and len(out['verify']) == 2, out
    # DDP at world 1 over RCCL (graphed) == the same training without DDP (eager)
    assert out['param_rel_diff'] < 1e-4, out
    assert out['max_loss_diff'] < 1e-3, out
