"""The ImageNet CLI with whole-step HIP graphs (``--graphs 1``) on the GPU:
K-FAC plain steps replayed, factor / second-order steps eager, and an eager
evaluation pass between epochs (the reference's epoch loop,
``examples/torch_imagenet_resnet.py:358-368``) -- the interleaving that
corrupted replays before the graph-safe strided convolutions
(distributed_kfac_pytorch_amd/ops/conv.py)."""
from __future__ import annotations

import pytest

from tests.test_examples import _run

pytestmark = pytest.mark.gpu


def test_imagenet_cli_graphs(tmp_path):
    err: list = []
    lines = _run(['examples/torch_imagenet_resnet.py', '--model', 'resnet50', '--epochs', '2',
                  '--image-size', '64', '--synthetic-train-size', '96',
                  '--synthetic-val-size', '32', '--batch-size', '8', '--val-batch-size', '8',
                  '--workers', '0', '--log-dir', str(tmp_path), '--kfac-inv-update-steps', '4',
                  '--kfac-factor-update-steps', '2', '--graphs', '1', '--checkpoint-freq', '2'], stderr=err)
    assert [line['epoch'] for line in lines] == [0, 1]
    for line in lines:
        assert line['train/loss'] == line['train/loss']  # not NaN
        assert line['val/loss'] == line['val/loss']
    # 12 steps per epoch: plain steps replayed from the captured graph
    assert lines[-1]['train/graph_replays'] >= 6, (lines[-1], err[0][-4000:])


def test_imagenet_cli_fp32_native_convs(tmp_path):
    """The bench's fp32 step from the CLI: native 1x1 and implicit-GEMM 3x3
    convolutions (``--conv1x1 gemm --conv-kxk gemm``) under whole-step
    graphs -- finite, replayed, and the capture-time check passed."""
    err: list = []
    lines = _run(['examples/torch_imagenet_resnet.py', '--model', 'resnet50', '--epochs', '1',
                  '--image-size', '64', '--synthetic-train-size', '96',
                  '--synthetic-val-size', '32', '--batch-size', '8', '--val-batch-size', '8',
                  '--workers', '0', '--log-dir', str(tmp_path), '--kfac-inv-update-steps', '4',
                  '--kfac-factor-update-steps', '2', '--graphs', '1', '--precision', 'fp32',
                  '--conv1x1', 'gemm', '--conv-kxk', 'gemm', '--checkpoint-freq', '5'],
                 stderr=err)
    assert [line['epoch'] for line in lines] == [0]
    assert lines[0]['train/loss'] == lines[0]['train/loss']
    assert lines[0]['val/loss'] == lines[0]['val/loss']
    assert lines[0]['train/graph_replays'] >= 3, (lines[0], err[0][-4000:])
