"""``bench.py --gpus N`` starts N ranks itself (CPU tests of the launcher).

The driver runs ``python bench.py --gpus 1`` and, for N > 1, wraps the same
script in ``torch.distributed.run``; a user running ``python bench.py --gpus
8`` directly must get 8 ranks too, not a silent world-1 run (reference
launcher: ``scripts/run_imagenet.sh:54-60``).
"""
from __future__ import annotations

import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def bench(monkeypatch):
    monkeypatch.syspath_prepend(ROOT)
    return importlib.import_module('bench')


def test_launcher_argv(bench) -> None:
    cmd = bench.launcher_argv(['--gpus', '4', '--steps', '3'], 4, 29555)
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=4' in cmd and '--nnodes=1' in cmd
    assert '--master-addr=127.0.0.1' in cmd and '--master-port=29555' in cmd
    i = cmd.index(os.path.join(ROOT, 'bench.py'))
    assert cmd[i + 1:] == ['--gpus', '4', '--steps', '3']


def test_world_guard(bench) -> None:
    bench.check_world(2, 2)
    with pytest.raises(SystemExit, match='--gpus 8 but the job has 1'):
        bench.check_world(1, 8)


def test_main_relaunches_without_world_size(bench, monkeypatch) -> None:
    seen = {}

    def fake_call(cmd):  # noqa: ANN001
        seen['cmd'] = cmd
        return 7

    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(subprocess, 'call', fake_call)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2', '--backend', 'gloo'])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7  # the child's exit status
    assert '--nproc-per-node=2' in seen['cmd']
    assert seen['cmd'][-4:] == ['--gpus', '2', '--backend', 'gloo']


def test_main_refuses_mismatched_world(bench, monkeypatch) -> None:
    monkeypatch.setenv('WORLD_SIZE', '1')
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2'])
    with pytest.raises(SystemExit, match='--gpus 2 but the job has 1'):
        bench.main()
