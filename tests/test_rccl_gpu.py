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
import re
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return int(s.getsockname()[1])


_CAUSE = re.compile(r'terminate called|what\(\)|Error|error:|Exception|Traceback|Fatal Python|'
                    r'File "|watchdog|SIGABRT|Signal \d+|HIP|hip[A-Z]\w+|RCCL WARN|NCCL WARN')


def diagnose(stdout: str, stderr: str, error_file: str) -> str:
    """The lines that name why a torchrun child failed: the rank's C++ abort
    message or Python traceback (faulthandler dumps every thread's stack on
    a fatal signal), RCCL warnings and torchrun's per-rank error file --
    not just the tail, which torchrun's summary fills."""
    keep = [ln for ln in (stdout + '\n' + stderr).splitlines() if _CAUSE.search(ln)]
    text = '\n'.join(keep[-80:])
    if os.path.exists(error_file):
        with open(error_file) as f:
            text += '\n--- torchelastic error file ---\n' + f.read()[-4000:]
    return text


def test_diagnose_keeps_abort_cause(tmp_path) -> None:
    err = "terminate called after throwing an instance of 'c10::DistBackendError'\n" \
          "  what():  Process group watchdog thread terminated with exception\n" + \
          'noise\n' * 500 + 'traceback : Signal 6 (SIGABRT) received by PID 1\n'
    f = tmp_path / 'err.json'
    f.write_text('{"message": "boom"}')
    d = diagnose('ok\n', err, str(f))
    assert 'watchdog thread terminated' in d and 'SIGABRT' in d and 'boom' in d
    assert 'noise' not in d


@pytest.mark.gpu
def test_ddp_kfac_graphs_over_rccl(cuda, tmp_path) -> None:
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    env['PYTHONUNBUFFERED'] = '1'
    error_file = str(tmp_path / 'torchelastic_error.json')
    env['TORCHELASTIC_ERROR_FILE'] = error_file
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=1',
           '--master-addr=127.0.0.1', f'--master-port={_port()}',
           os.path.join(ROOT, 'tests', '_rccl_worker.py')]
    proc = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    log = tmp_path / 'rccl_worker.log'
    log.write_text(f'rc={proc.returncode}\n--- stdout ---\n{proc.stdout}\n'
                   f'--- stderr ---\n{proc.stderr}\n')
    keep = os.environ.get('KFAC_TEST_LOG_DIR')
    if keep:  # a copy that outlives pytest's tmp dir (gpurun_out/ on the box)
        os.makedirs(keep, exist_ok=True)
        with open(os.path.join(keep, 'rccl_worker.log'), 'w') as f:
            f.write(log.read_text())
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith('RESULT ')]
    assert proc.returncode == 0 and lines, (
        f'torchrun rc={proc.returncode}; full log {log}\n'
        + diagnose(proc.stdout, proc.stderr, error_file))
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
