"""Multi-process test harness (the role of reference ``testing/distributed.py``).

``@distributed_test(world_size)`` runs the decorated test body in
``world_size`` forked processes joined by a gloo process group on
127.0.0.1, with a hang timeout.  A list of world sizes runs the body once
per size.  Each run gets a fresh port so consecutive tests never collide.
"""
from __future__ import annotations

import functools
import multiprocessing as mp
import os
import socket
import traceback
from typing import Any
from typing import Callable

import torch.distributed as dist

TIMEOUT_S = 60.0


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return int(s.getsockname()[1])


def _worker(rank: int, world: int, port: int, fn: Callable[..., Any],
            args: tuple, kwargs: dict, errq: Any) -> None:
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['RANK'] = str(rank)
    os.environ['LOCAL_RANK'] = str(rank)
    os.environ['WORLD_SIZE'] = str(world)
    try:
        dist.init_process_group('gloo', rank=rank, world_size=world)
        fn(*args, **kwargs)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:  # noqa: BLE001
        errq.put((rank, traceback.format_exc()))
        errq.close()
        errq.join_thread()
        os._exit(1)
    os._exit(0)


def run_distributed(fn: Callable[..., Any], world_size: int, *args: Any, **kwargs: Any) -> None:
    ctx = mp.get_context('fork')
    errq = ctx.Queue()
    port = _free_port()
    procs = [
        ctx.Process(target=_worker, args=(r, world_size, port, fn, args, kwargs, errq))
        for r in range(world_size)
    ]
    for p in procs:
        p.start()
    failures = []
    for p in procs:
        p.join(TIMEOUT_S)
    for r, p in enumerate(procs):
        if p.is_alive():
            p.terminate()
            p.join(5)
            failures.append(f'rank {r} hung (>{TIMEOUT_S}s)')
        elif p.exitcode != 0:
            failures.append(f'rank {r} exited with {p.exitcode}')
    errors = []
    while not errq.empty():
        errors.append(errq.get())
    if failures or errors:
        msg = '\n'.join(failures)
        for r, tb in sorted(errors):
            msg += f'\n--- rank {r} ---\n{tb}'
        raise AssertionError(msg)


def distributed_test(world_size: int | list[int] = 2) -> Callable:
    sizes = [world_size] if isinstance(world_size, int) else list(world_size)

    def deco(fn: Callable) -> Callable:
        @functools.wraps(fn)
        def wrapper(*args: Any, **kwargs: Any) -> None:
            for w in sizes:
                run_distributed(fn, w, *args, **kwargs)

        return wrapper

    return deco
