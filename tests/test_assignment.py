"""KAISA placement (reference tests/assignment_test.py strategy: N ranks are
simulated by building N assignment objects in one process)."""
from __future__ import annotations

import pytest

from distributed_kfac_pytorch_amd.parallel.assignment import KAISAAssignment


def identity(ranks):
    return ranks


@pytest.mark.parametrize(
    'world,gw,cols,rows',
    [
        (1, 1, [[0]], [[0]]),
        (2, 1, [[0], [1]], [[0, 1]]),
        (2, 2, [[0, 1]], [[0], [1]]),
        (8, 2, [[0, 4], [1, 5], [2, 6], [3, 7]], [[0, 1, 2, 3], [4, 5, 6, 7]]),
        (8, 4, [[0, 2, 4, 6], [1, 3, 5, 7]], [[0, 1], [2, 3], [4, 5], [6, 7]]),
        (16, 8, [list(range(0, 16, 2)), list(range(1, 16, 2))],
         [[2 * i, 2 * i + 1] for i in range(8)]),
    ],
)
def test_partitions(world, gw, cols, rows):
    c = KAISAAssignment.partition_grad_workers(world, gw)
    r = KAISAAssignment.partition_grad_receivers(world, gw)
    assert sorted(sorted(x) for x in c) == sorted(cols)
    assert sorted(sorted(x) for x in r) == sorted(rows)


def test_partition_validation():
    with pytest.raises(ValueError):
        KAISAAssignment.partition_grad_workers(0, 1)
    with pytest.raises(ValueError):
        KAISAAssignment.partition_grad_workers(8, 3)
    with pytest.raises(ValueError):
        KAISAAssignment.partition_grad_receivers(8, 3)


def test_constructor_validation():
    work = {'l': {'A': 1.0, 'G': 1.0}}
    with pytest.raises(ValueError):
        KAISAAssignment(work, local_rank=0, world_size=2, grad_worker_fraction=2,
                        group_func=identity)
    with pytest.raises(ValueError):
        KAISAAssignment(work, local_rank=-1, world_size=2, grad_worker_fraction=1,
                        group_func=identity)
    with pytest.raises(ValueError):
        KAISAAssignment(work, local_rank=2, world_size=2, grad_worker_fraction=1,
                        group_func=identity)
    with pytest.raises(ValueError):  # 8 * 0.3 not an integer
        KAISAAssignment(work, local_rank=0, world_size=8, grad_worker_fraction=0.3,
                        group_func=identity)


@pytest.mark.parametrize(
    'world,frac,expected',
    [(1, 1.0, 1), (1, 0.5, 1), (4, 0.25, 1), (4, 0.5, 2), (4, 1.0, 4), (8, 0.0, 1)],
)
def test_grad_worker_count(world, frac, expected):
    a = KAISAAssignment({'l': {'A': 1, 'G': 1}}, local_rank=0, world_size=world,
                        grad_worker_fraction=frac, group_func=identity)
    assert a.grad_workers == expected
    assert a.broadcast_gradients() == (expected < world)
    assert a.broadcast_inverses() == (expected > 1)


def test_greedy_colocated():
    work = {
        'l1': {'A': 1, 'G': 1},
        'l2': {'A': 2, 'G': 2},
        'l3': {'A': 3, 'G': 3},
    }
    got = KAISAAssignment.greedy_assignment(work, [[0], [1]], 2, True)
    assert got == {
        'l1': {'A': 1, 'G': 1},
        'l2': {'A': 1, 'G': 1},
        'l3': {'A': 0, 'G': 0},
    }


def test_greedy_not_colocated():
    work = {'l1': {'A': 5, 'G': 1}, 'l2': {'A': 2, 'G': 3}}
    got = KAISAAssignment.greedy_assignment(work, [[0, 1]], 2, False)
    assert got == {'l1': {'A': 0, 'G': 1}, 'l2': {'A': 1, 'G': 1}}


def test_greedy_groups_balance():
    # 4 equal layers over 2 columns of 2 ranks: one layer per rank
    work = {f'l{i}': {'A': 1, 'G': 1} for i in range(4)}
    got = KAISAAssignment.greedy_assignment(work, [[0, 2], [1, 3]], 4, True)
    ranks = sorted(v['A'] for v in got.values())
    assert ranks == [0, 1, 2, 3]
    for v in got.values():
        assert v['A'] == v['G']


@pytest.mark.parametrize('world,frac', [(1, 1.0), (2, 0.5), (4, 0.5), (8, 0.5), (8, 0.25), (8, 1.0), (8, 0.125)])
@pytest.mark.parametrize('colocate', [True, False])
def test_simulated_ranks_agree(world, frac, colocate):
    work = {f'layer{i}': {'A': float((i * 7) % 13 + 1) ** 3, 'G': float((i * 5) % 11 + 1) ** 3}
            for i in range(20)}
    assigns = [
        KAISAAssignment(work, local_rank=r, world_size=world,
                        grad_worker_fraction=frac, group_func=identity,
                        colocate_factors=colocate)
        for r in range(world)
    ]
    gw = max(1, int(world * frac))
    for layer in work:
        invs = {(a.inv_worker(layer, 'A'), a.inv_worker(layer, 'G')) for a in assigns}
        assert len(invs) == 1
        if colocate:
            ia, ig = invs.pop()
            assert ia == ig
        workers = [r for r, a in enumerate(assigns) if a.is_grad_worker(layer)]
        assert len(workers) == gw
        for a in assigns:
            # inverse worker belongs to the grad worker group
            assert a.inv_worker(layer, 'A') in workers
            assert sorted(a.grad_worker_group(layer)) == workers
            src = a.src_grad_worker(layer)
            assert src in workers
            assert a.local_rank in a.grad_receiver_group(layer)
            assert src in a.grad_receiver_group(layer)
            if a.is_grad_worker(layer):
                assert src == a.local_rank
            assert a.factor_group(layer, 'A') is None
        # one source per receiver row
        srcs = {a.src_grad_worker(layer) for a in assigns}
        assert len(srcs) == gw


def test_groups_created_once_in_order():
    calls = []

    def record(ranks):
        calls.append(tuple(ranks))
        return tuple(ranks)

    KAISAAssignment({'l': {'A': 1, 'G': 1}}, local_rank=3, world_size=8,
                    grad_worker_fraction=0.5, group_func=record)
    assert calls == [
        (0, 2, 4, 6), (1, 3, 5, 7), (0, 1), (2, 3), (4, 5), (6, 7),
    ]


def test_repr_lists_layers():
    a = KAISAAssignment({'x': {'A': 1, 'G': 2}}, local_rank=0, world_size=1,
                        grad_worker_fraction=1.0, group_func=identity)
    s = repr(a)
    assert 'layer="x"' in s and 'inv_workers' in s


def _expectation_cases() -> list:
    import json
    import os

    path = os.path.join(os.path.dirname(__file__), 'data', 'assignment_expectations.json')
    with open(path) as f:
        return [pytest.param(*c[1:], id=c[0]) for c in json.load(f)['cases']]


@pytest.mark.parametrize(
    'work,worker_groups,world_size,colocate,expected', _expectation_cases(),
)
def test_greedy_assignment_reference_table(work, worker_groups, world_size, colocate,
                                           expected):
    """The reference's exact greedy placements, including its tie-break
    order (descending cost, then descending key), pinned as data."""
    from distributed_kfac_pytorch_amd.parallel.assignment import KAISAAssignment

    assert KAISAAssignment.greedy_assignment(
        work, worker_groups, world_size, colocate,
    ) == expected
