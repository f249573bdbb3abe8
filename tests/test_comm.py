"""Collectives (reference tests/distributed_test.py strategy; gloo on CPU)."""
from __future__ import annotations

import pytest
import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.parallel.comm import AllreduceTensorBucket
from distributed_kfac_pytorch_amd.parallel.comm import AsyncTensor
from distributed_kfac_pytorch_amd.parallel.comm import fill_triu
from distributed_kfac_pytorch_amd.parallel.comm import get_rank
from distributed_kfac_pytorch_amd.parallel.comm import get_triu
from distributed_kfac_pytorch_amd.parallel.comm import get_world_size
from distributed_kfac_pytorch_amd.parallel.comm import NonSquareTensorError
from distributed_kfac_pytorch_amd.parallel.comm import TorchDistributedCommunicator
from tests.harness import distributed_test


@pytest.mark.parametrize('shape', [(1, 1), (5, 5), (3, 7)])
def test_triu_roundtrip(shape):
    t = torch.randn(*shape)
    tri = get_triu(t)
    idx = torch.triu_indices(*shape)
    assert torch.equal(tri, t[idx[0], idx[1]])
    if shape[0] == shape[1]:
        s = t + t.t()
        assert torch.equal(fill_triu(shape, get_triu(s)), s)


def test_triu_errors():
    with pytest.raises(ValueError):
        get_triu(torch.zeros(3))
    with pytest.raises(ValueError):
        get_triu(torch.zeros(4, 2))
    with pytest.raises(ValueError):
        fill_triu((3,), torch.zeros(3))


def test_non_distributed_defaults():
    assert get_rank() == 0
    assert get_world_size() == 1
    tdc = TorchDistributedCommunicator()
    t = torch.ones(3)
    assert tdc.allreduce(t) is t
    assert tdc.broadcast(t, src=0) is t
    assert tdc.allreduce_bucketed(t) is t
    assert tdc.bucket_cap_bytes == 25_000_000


def test_async_tensor_resolves_once():
    calls = []

    def fin():
        calls.append(1)
        return torch.ones(2)

    a = AsyncTensor(finalize=fin)
    assert not a.done()
    assert torch.equal(a.wait(), torch.ones(2))
    a.wait()
    assert calls == [1] and a.done()


@distributed_test([1, 4])
def _allreduce_body():
    world = dist.get_world_size()
    rank = dist.get_rank()
    tdc = TorchDistributedCommunicator()
    for symmetric in (False, True):
        base = torch.arange(16.0).reshape(4, 4)
        base = base + base.t()
        t = base.clone() * (rank + 1)
        out = tdc.allreduce(t, symmetric=symmetric)
        out = out.wait() if isinstance(out, AsyncTensor) else out
        assert torch.allclose(out, base * sum(range(1, world + 1)))
        t = base.clone() * (rank + 1)
        out = tdc.allreduce(t, average=True, symmetric=symmetric)
        out = out.wait() if isinstance(out, AsyncTensor) else out
        assert torch.allclose(out, base * sum(range(1, world + 1)) / world)
    if world > 1:
        with pytest.raises(NonSquareTensorError):
            tdc.allreduce(torch.ones(2, 3), symmetric=True)
        with pytest.raises(NonSquareTensorError):
            tdc.broadcast(torch.ones(2, 3), src=0, symmetric=True)


def test_allreduce():
    _allreduce_body()


@distributed_test([1, 4])
def _broadcast_body():
    rank = dist.get_rank()
    tdc = TorchDistributedCommunicator()
    for symmetric in (False, True):
        base = torch.randn(5, 5, generator=torch.Generator().manual_seed(7))
        base = base + base.t()
        t = base.clone() if rank == 0 else torch.zeros(5, 5)
        out = tdc.broadcast(t, src=0, symmetric=symmetric)
        out = out.wait() if isinstance(out, AsyncTensor) else out
        assert torch.allclose(out, base)


def test_broadcast():
    _broadcast_body()


def test_bucket_semantics():
    b = AllreduceTensorBucket()
    assert b.size == 0 and not b.communicated()
    b.add_tensor(torch.ones(10))
    assert b.size == 40
    b.add_tensor(torch.ones(3, 3), symmetric=True)
    assert b.size == 40 + 6 * 4


@distributed_test(4)
def _bucket_body():
    world = dist.get_world_size()
    b = AllreduceTensorBucket()
    ts = [torch.ones(4) * (i + 1) for i in range(3)]
    futs = [b.add_tensor(t) for t in ts]
    b.allreduce()
    with pytest.raises(RuntimeError):
        b.allreduce()
    for i, f in enumerate(futs):
        assert torch.allclose(f.wait(), torch.ones(4) * (i + 1) * world)


def test_bucket_allreduce():
    _bucket_body()


@distributed_test(4)
def _bucketed_body():
    world = dist.get_world_size()
    rank = dist.get_rank()
    # cap of 1e-4 MB = 100 bytes: small tensors share buckets, a big one is
    # alone in its own bucket
    tdc = TorchDistributedCommunicator(bucket_cap_mb=1e-4)
    sizes = [(2, 2), (3, 3), (20, 20), (2, 2), (4, 4)]
    inputs = []
    handles = []
    for i, s in enumerate(sizes):
        base = torch.randn(*s, generator=torch.Generator().manual_seed(i))
        base = base + base.t()
        inputs.append(base)
        t = base.clone() * (rank + 1)
        handles.append(tdc.allreduce_bucketed(t, average=(i % 2 == 0), symmetric=(i % 3 == 0)))
    tdc.flush_allreduce_buckets()
    total = sum(range(1, world + 1))
    for i, (h, base) in enumerate(zip(handles, inputs)):
        out = h.wait()
        expect = base * total / (world if i % 2 == 0 else 1)
        assert torch.allclose(out, expect, atol=1e-5), i


def test_allreduce_bucketed():
    _bucketed_body()


@distributed_test(4)
def _subgroup_body():
    rank = dist.get_rank()
    group = dist.new_group([1, 2, 3])
    tdc = TorchDistributedCommunicator(bucket_cap_mb=1)
    if rank != 0:
        t = torch.ones(3, 3) * rank
        h = tdc.allreduce_bucketed(t, group=group, average=True)
        tdc.flush_allreduce_buckets()
        assert torch.allclose(h.wait(), torch.ones(3, 3) * 2.0)
        assert tdc.group_ranks(group) == frozenset({1, 2, 3})
    else:
        tdc.flush_allreduce_buckets()


def test_subgroup_buckets():
    _subgroup_body()


@distributed_test(2)
def _bcast_bucket_body():
    rank = dist.get_rank()
    tdc = TorchDistributedCommunicator(bucket_cap_mb=1e-4)  # 100 bytes
    shapes = [(2, 3), (4, 4), (10, 10), (1, 5)]
    srcs = [0, 1, 0, 1]
    handles, expect = [], []
    for i, (s, src) in enumerate(zip(shapes, srcs)):
        val = torch.full(s, float(i + 10 * src))
        t = val.clone() if rank == src else torch.zeros(s)
        handles.append(tdc.broadcast_bucketed(t, src=src))
        expect.append(val)
    tdc.flush_broadcast_buckets()
    for h, e in zip(handles, expect):
        out = h.wait() if isinstance(h, AsyncTensor) else h
        assert torch.equal(out, e)


def test_broadcast_bucketed():
    _bcast_bucket_body()


@distributed_test(4)
def _exchange_bucket_body():
    """Per-group gradient exchange (one all-gather per receiver group):
    every member is the source of some tensors, shares are uneven, the cap
    splits the bucket, and receivers get exactly the source's values."""
    rank = dist.get_rank()
    # two receiver groups {0, 1} and {2, 3} (KAISA rows at world 4, gwf 0.5)
    groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
    group = groups[rank // 2]
    base = 2 * (rank // 2)
    tdc = TorchDistributedCommunicator(bucket_cap_mb=3e-4)  # 300 bytes per member
    shapes = [(2, 3), (4, 4), (10, 10), (1, 5), (7,), (3, 3)]
    srcs = [base + s for s in (0, 1, 0, 0, 1, 1)]
    handles, expect = [], []
    for i, (shape, src) in enumerate(zip(shapes, srcs)):
        val = torch.full(shape, float(i + 10 * src)) + torch.arange(
            torch.Size(shape).numel(), dtype=torch.float32).view(shape)
        t = val.clone() if rank == src else torch.full(shape, -1.0)
        handles.append(tdc.exchange_bucketed(t, src=src, group=group))
        expect.append(val)
    tdc.flush_broadcast_buckets()
    for h, e in zip(handles, expect):
        out = h.wait() if isinstance(h, AsyncTensor) else h
        assert torch.equal(out, e)


def test_exchange_bucketed():
    _exchange_bucket_body()
