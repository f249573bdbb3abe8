"""Example CLIs run end to end on the CPU (synthetic data, gloo).

Each CLI runs in a subprocess (it creates its own process group); the
2-rank case goes through ``torch.distributed.run`` exactly like a GPU node
launch, at 127.0.0.1.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from examples.vision.optimizers import milestone_lambda

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _env() -> dict[str, str]:
    env = dict(os.environ)
    env['PYTHONPATH'] = ROOT + os.pathsep + env.get('PYTHONPATH', '')
    env['OMP_NUM_THREADS'] = '1'
    env['MASTER_ADDR'] = '127.0.0.1'
    env['MASTER_PORT'] = str(_port())
    env.pop('RANK', None)
    env.pop('WORLD_SIZE', None)
    env.pop('LOCAL_RANK', None)
    return env


def _run(args: list[str], nproc: int = 1, timeout: int = 240,
         stderr: list | None = None) -> list[dict]:
    """Run a CLI; returns its JSON log lines (``stderr`` collects its stderr)."""
    env = _env()
    if nproc > 1:
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
               f'--nproc-per-node={nproc}', '--master-addr', '127.0.0.1',
               '--master-port', env['MASTER_PORT']] + args
    else:
        cmd = [sys.executable] + args
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    if stderr is not None:
        stderr.append(p.stderr)
    out = []
    for line in p.stdout.splitlines():
        if line.startswith('{'):
            out.append(json.loads(line))
    return out


def test_milestone_lambda_does_not_compound():
    f = milestone_lambda(0.5, [2, 4])
    assert [f(e) for e in range(6)] == [1, 1, 0.5, 1, 0.5, 1]


@pytest.mark.parametrize('nproc,extra', [
    (1, []),
    (2, ['--kfac-strategy', 'hybrid-opt', '--kfac-grad-worker-fraction', '0.5',
         '--batches-per-allreduce', '2']),
])
def test_cifar10_cli(tmp_path, nproc, extra):
    args = ['examples/torch_cifar10_resnet.py', '--model', 'resnet20', '--epochs', '2',
            '--synthetic-train-size', '256', '--synthetic-val-size', '64',
            '--batch-size', '32', '--val-batch-size', '32', '--workers', '0',
            '--log-dir', str(tmp_path), '--kfac-inv-update-steps', '2',
            '--checkpoint-freq', '1', '--no-cuda'] + extra
    lines = _run(args, nproc)
    assert [line['epoch'] for line in lines] == [0, 1]
    assert all(line['train/loss'] == line['train/loss'] for line in lines)  # not NaN
    assert (tmp_path / 'checkpoint_2.pth.tar').exists()
    # auto-resume picks up epoch 2 and trains one more epoch
    lines = _run([a if a != '2' or i != 4 else '3' for i, a in enumerate(args)], nproc)
    assert [line['epoch'] for line in lines] == [2]


def test_imagenet_cli_small(tmp_path):
    lines = _run(['examples/torch_imagenet_resnet.py', '--model', 'resnet18', '--epochs', '1',
                  '--image-size', '64', '--synthetic-train-size', '32',
                  '--synthetic-val-size', '16', '--batch-size', '8', '--val-batch-size', '8',
                  '--workers', '0', '--log-dir', str(tmp_path), '--kfac-inv-update-steps', '2',
                  '--kfac-factor-update-steps', '1', '--no-cuda'])
    assert lines[-1]['epoch'] == 0
    assert (tmp_path / 'scalars.jsonl').exists() or any(tmp_path.iterdir())


def test_imagenet_cli_sgd_only(tmp_path):
    lines = _run(['examples/torch_imagenet_resnet.py', '--model', 'resnet18', '--epochs', '1',
                  '--image-size', '32', '--synthetic-train-size', '16',
                  '--synthetic-val-size', '8', '--batch-size', '8', '--workers', '0',
                  '--log-dir', str(tmp_path), '--kfac-inv-update-steps', '0', '--no-cuda'])
    assert lines[-1]['epoch'] == 0


@pytest.mark.parametrize('nproc', [1, 2])
def test_language_model_cli(nproc):
    lines = _run(['examples/torch_language_model.py', '--kfac', '--epochs', '2',
                  '--synthetic-tokens', '8000', '--max-steps-per-epoch', '6',
                  '--embedding-dim', '32', '--hidden-dim', '32', '--inv-update-steps', '2',
                  '--register-embeddings', '--skip-layers', 'decoder', 'self_attn',
                  '--strategy', 'mem_opt', '--backend', 'gloo', '--no-cuda'], nproc)
    assert [line['epoch'] for line in lines] == [1, 2]


def test_gpt_neox_cli_tp(tmp_path):
    lines = _run(['examples/torch_gpt_neox.py', '--mp', '2', '--steps', '4', '--seq-len', '16',
                  '--micro-batch', '2', '--factor-update-steps', '1', '--inv-update-steps', '2',
                  '--log-interval', '2', '--no-cuda', '--backend', 'gloo',
                  '--factor-checkpoint-dir', str(tmp_path)], nproc=4)
    assert [line['step'] for line in lines if 'step' in line] == [2, 4]
    assert lines[-1]['tokens_per_s'] > 0
    assert len(list(tmp_path.iterdir())) == 8  # one factor file per TP layer


def test_gpt_neox_cli_pipeline(tmp_path):
    """pp 2 x mp 2 (4 gloo ranks): GPipe schedule, K-FAC per stage."""
    lines = _run(['examples/torch_gpt_neox.py', '--pp', '2', '--mp', '2', '--micro-batches', '2',
                  '--steps', '4', '--seq-len', '16', '--micro-batch', '4',
                  '--factor-update-steps', '1', '--inv-update-steps', '2',
                  '--log-interval', '2', '--no-cuda', '--backend', 'gloo'], nproc=4)
    assert [line['step'] for line in lines if 'step' in line] == [2, 4]
    assert lines[-1]['tokens_per_s'] > 0
