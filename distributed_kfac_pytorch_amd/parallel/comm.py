"""K-FAC collectives over ``torch.distributed`` (RCCL on MI355X, gloo on CPU).

Parity target: reference ``kfac/distributed.py:35-459``
(``TorchDistributedCommunicator``, ``AllreduceTensorBucket``, ``get_triu``,
``fill_triu``, ``get_rank``, ``get_world_size``, ``NonSquareTensorError``).

MI355X-first design differences (behaviour visible to callers is the same):

* No ``torch.futures`` callbacks.  A collective returns an ``AsyncTensor``:
  the RCCL ``Work`` handle plus a *finalize* step.  ``AsyncTensor.wait()``
  calls ``Work.wait()`` -- on RCCL this only makes the current HIP stream wait
  on RCCL's stream (the host does not block) -- and then enqueues the
  finalize (average scaling, upper-triangle unpack) on the current stream.
  The finalize writes back IN PLACE into the caller's tensor, so a factor
  keeps one device allocation for its whole life.
* Symmetric (upper-triangle) packing and unpacking, and the flat-bucket
  pack/unpack, are native HIP kernels (``ops.comm_pack``) on GPU tensors: one
  launch per bucket instead of a gather/scatter pair per tensor.
* Buckets are keyed by the process group object (the reference keys them by
  group *size*, ``distributed.py:370-372``, which lets two different
  same-size groups share a bucket; that quirk is deliberately fixed).
* Factor all-reduce without pack / unpack passes (``PackedFactorBuffer``):
  on GPU, a symmetric factor reduced over a group of more than one rank
  lives, between second-order updates, as its packed upper triangle inside
  ONE persistent per-group buffer.  The factor-update SYRK reads the
  averaged triangle from its slot and writes the new local value there
  pre-scaled by 1/world (csrc/syrk.hip packed epilogue), so the all-reduce
  (sum) of the buffer IS the averaged factor: no pack kernel before the
  collective, no unpack after it, no per-step bucket allocation.  The dense
  matrix is materialised (one unpack) only when something reads the factor
  -- the eigendecomposition / inversion every ``inv_update_steps`` steps,
  checkpointing.
"""
from __future__ import annotations

import collections
from typing import Any
from typing import Callable
from typing import Union

import torch
import torch.distributed as dist

from distributed_kfac_pytorch_amd.ops import comm_pack


class NonSquareTensorError(Exception):
    """Raised when a symmetric collective gets a non-square tensor."""


def get_rank(group: dist.ProcessGroup | None = None) -> int:
    """Rank in ``group`` (global rank if None); 0 without torch.distributed."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group)
    return 0


def get_world_size(group: dist.ProcessGroup | None = None) -> int:
    """Size of ``group`` (world if None); 1 without torch.distributed."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def get_triu(tensor: torch.Tensor) -> torch.Tensor:
    """Row-major flattened upper triangle (incl. diagonal) of a 2D tensor."""
    if tensor.dim() != 2:
        raise ValueError('triu(tensor) requires tensor to be 2 dimensional')
    if tensor.shape[0] > tensor.shape[1]:
        raise ValueError('tensor cannot have more rows than columns')
    return comm_pack.triu_pack(tensor)


def fill_triu(
    shape: tuple[int, ...] | torch.Size | list[int],
    triu_tensor: torch.Tensor,
) -> torch.Tensor:
    """Rebuild the symmetric matrix whose ``get_triu`` is ``triu_tensor``."""
    if len(shape) != 2:
        raise ValueError('shape must be 2 dimensional')
    rows, cols = int(shape[0]), int(shape[1])
    out = triu_tensor.new_empty((rows, cols))
    comm_pack.triu_unpack_(out, triu_tensor, 1.0)
    return out


class AsyncTensor:
    """Result of an asynchronous K-FAC collective.

    ``wait()`` returns the finished tensor.  It is idempotent.  The object is
    what the reference exposes as a ``torch.futures.Future``; the layer
    properties resolve it lazily in the same way
    (reference ``kfac/layers/base.py:93-127``).
    """

    __slots__ = ('_work', '_finalize', '_result', '_done', '_bucket')

    def __init__(
        self,
        work: Any | None = None,
        finalize: Callable[[], torch.Tensor] | None = None,
        result: torch.Tensor | None = None,
        bucket: AllreduceTensorBucket | None = None,
    ) -> None:
        self._work = work
        self._finalize = finalize
        self._result = result
        self._done = finalize is None and bucket is None
        self._bucket = bucket

    def done(self) -> bool:
        return self._done

    def wait(self) -> torch.Tensor:
        if self._done:
            assert self._result is not None
            return self._result
        if self._bucket is not None:
            if not self._bucket.communicated():
                raise RuntimeError(
                    'waiting on a tensor whose all-reduce bucket was never '
                    'launched; call flush_allreduce_buckets() on every rank',
                )
            self._work = self._bucket.work
            self._bucket = None
        if self._work is not None:
            self._work.wait()
        assert self._finalize is not None
        self._result = self._finalize()
        self._finalize = None
        self._work = None
        self._done = True
        return self._result

    # torch.futures.Future-like aliases used by some callers
    def value(self) -> torch.Tensor:
        return self.wait()


# What layer state may hold while a collective is in flight.
Future = (AsyncTensor,)
FutureType = Union[AsyncTensor]


def _result_buffer(
    tensor: torch.Tensor,
    wire: torch.Tensor,
    symmetric: bool,
) -> torch.Tensor:
    """Where a collective's result lands: the caller's tensor when it is
    contiguous (in place), else the contiguous wire buffer, or a fresh
    dense matrix for a triangle-packed wire."""
    if tensor.is_contiguous():
        return tensor
    if symmetric:
        return torch.empty_like(tensor, memory_format=torch.contiguous_format)
    return wire


def _scale_for(average: bool, group: dist.ProcessGroup | None) -> float:
    return 1.0 / get_world_size(group) if average else 1.0


class AllreduceTensorBucket:
    """A fused all-reduce of several tensors through one flat buffer."""

    def __init__(
        self,
        group: dist.ProcessGroup | None = None,
    ) -> None:
        self._group = group
        self._entries: list[tuple[torch.Tensor, bool]] = []
        self._slots: list[AsyncTensor] = []
        self._size = 0
        self._communicated = False
        self.work: Any | None = None
        self.flat: torch.Tensor | None = None

    @property
    def size(self) -> int:
        """Bytes currently in the bucket (after triangle packing)."""
        return self._size

    def communicated(self) -> bool:
        return self._communicated

    def add_tensor(
        self,
        tensor: torch.Tensor,
        *,
        symmetric: bool = False,
        finalize: Callable[[torch.Tensor], torch.Tensor] | None = None,
    ) -> AsyncTensor:
        """Queue ``tensor``; the returned handle resolves to its reduced value.

        ``symmetric`` packs only the upper triangle into the bucket.  The
        handle's value is, by default, a view of the reduced flat buffer
        (reshaped, or triangle-unpacked into a new tensor); ``finalize`` can
        override how the reduced slice is turned into the result.
        """
        if self._communicated:
            raise RuntimeError('bucket was already communicated')
        n = comm_pack.packed_numel(tensor, symmetric)
        offset = sum(comm_pack.packed_numel(t, s) for t, s in self._entries)
        self._entries.append((tensor, symmetric))
        self._size += n * tensor.element_size()

        def _finish() -> torch.Tensor:
            assert self.flat is not None
            sl = self.flat[offset: offset + n]
            if finalize is not None:
                return finalize(sl)
            if symmetric:
                return fill_triu(tensor.shape, sl)
            return sl.view(tensor.shape)

        slot = AsyncTensor(finalize=_finish, bucket=self)
        self._slots.append(slot)
        return slot

    def allreduce(self) -> Any | None:
        """Pack, launch the all-reduce, and return its ``Work`` (or None)."""
        if self._communicated:
            raise RuntimeError(
                'Communication for this bucket has already been performed. '
                'Ensure allreduce() is only called once for a given bucket.',
            )
        self._communicated = True
        if not self._entries:
            return None
        total = sum(comm_pack.packed_numel(t, s) for t, s in self._entries)
        ref = self._entries[0][0]
        # A fresh flat buffer per bucket: the caching allocator makes this
        # free in steady state, and RCCL's stream is recorded on it so the
        # memory is not recycled before the collective finishes.
        self.flat = torch.empty(total, dtype=ref.dtype, device=ref.device)
        comm_pack.pack_flat(self.flat, self._entries)
        self.work = dist.all_reduce(self.flat, group=self._group, async_op=True)
        return self.work


class PackedFactorBuffer:
    """Persistent all-reduce buffer of the packed factor triangles of one
    process group (see the module docstring).

    Layout: the preconditioner ``reserve()``s every factor of the group once,
    before the first factor update -- A factors in forward order, then G
    factors in backward order, i.e. the order the hooks produce them -- and
    the buffer is allocated ONCE at its final size.  A factor that was not
    reserved still gets a slot on first use (the buffer is then re-allocated
    and copied, after waiting for every collective in flight); slots never
    move otherwise.  The layout is identical on every rank: every rank
    registers the same layers in the same order.

    Launch: the buffer is cut into contiguous cap-sized chunks.  With
    ``eager_launch`` (default; ``KFAC_PACKED_EAGER_LAUNCH=0`` turns it off) a
    chunk is all-reduced from ``mark()`` -- i.e. from the forward / backward
    hook, on the stream that just wrote the slot -- as soon as EVERY slot of
    the chunk has been marked, so the factor all-reduce overlaps the rest of
    forward / backward as the reference's hook-launched buckets do
    (``kfac/distributed.py:299-368``, ``kfac/base_preconditioner.py:450-477``).
    ``launch()`` (from ``step()``) all-reduces the chunks still holding marked
    slots.  Chunks complete in hook order, which is the same on every rank,
    so every rank issues the same collective sequence.
    """

    def __init__(self, group: dist.ProcessGroup | None, cap_bytes: int,
                 eager_launch: bool | None = None) -> None:
        self.group = group
        self._cap = cap_bytes
        self._slots: dict[Any, tuple[int, int]] = {}
        self._size = 0
        self.flat: torch.Tensor | None = None
        self._chunks: list[tuple[int, int, list[Any]]] = []
        self._chunk_of: dict[Any, int] = {}
        self._dirty: list[Any] = []
        self._marked: dict[int, set] = {}
        self._works: dict[Any, Any] = {}
        if eager_launch is None:
            import os

            eager_launch = os.environ.get('KFAC_PACKED_EAGER_LAUNCH', '1') != '0'
        self.eager_launch = eager_launch
        self.launches = 0
        self.allocations = 0
        # (chunk index, 'hook' | 'step') of the latest chunk all-reduces
        self.launch_log: collections.deque = collections.deque(maxlen=4096)

    def reserve(self, layout: list[tuple[Any, int]], dtype: torch.dtype,
                device: torch.device) -> None:
        """Assign every slot of ``layout`` (``(key, numel)`` in hook order)
        and allocate the buffer once.  A no-op once the buffer exists."""
        if self.flat is not None or not layout:
            return
        for key, n in layout:
            if key not in self._slots:
                self._slots[key] = (self._size, int(n))
                self._size += int(n)
        self.flat = torch.zeros(self._size, dtype=dtype, device=device)
        self.allocations += 1
        self._rechunk()

    def _rechunk(self) -> None:
        self._chunks = []
        self._chunk_of = {}
        start = end = 0
        keys: list[Any] = []
        item = self.flat.element_size() if self.flat is not None else 4
        for key, (off, n) in sorted(self._slots.items(), key=lambda kv: kv[1][0]):
            if keys and self._cap > 0 and (end + n - start) * item > self._cap:
                self._chunks.append((start, end, keys))
                start, keys = end, []
            keys.append(key)
            end = off + n
            if self._cap <= 0:  # unbucketed: one collective per factor
                self._chunks.append((start, end, keys))
                start, keys = end, []
        if keys:
            self._chunks.append((start, end, keys))
        for i, (_, _, ks) in enumerate(self._chunks):
            for k in ks:
                self._chunk_of[k] = i

    def has(self, key: Any) -> bool:
        return key in self._slots

    def view(self, key: Any, numel: int | None = None, like: torch.Tensor | None = None) -> torch.Tensor:
        """The slot of ``key`` (registered on first use with ``numel``
        elements of ``like``'s dtype / device)."""
        if key not in self._slots:
            assert numel is not None and like is not None
            for w in self._works.values():
                if w is not None:
                    w.wait()
            self._works = {}
            old = self.flat
            self._slots[key] = (self._size, numel)
            self._size += numel
            self.flat = torch.zeros(self._size, dtype=like.dtype, device=like.device)
            self.allocations += 1
            if old is not None:
                self.flat[: old.numel()].copy_(old)
            self._rechunk()
            self._marked = {}
            for k in self._dirty:
                self._marked.setdefault(self._chunk_of[k], set()).add(k)
        off, n = self._slots[key]
        assert self.flat is not None
        return self.flat[off: off + n]

    def mark(self, key: Any) -> None:
        """The slot holds a new pre-scaled local value to be summed.  With
        ``eager_launch``, all-reduce its chunk now if this completes it
        (collective: every rank marks the same keys in the same order)."""
        if key in self._dirty:
            return
        self._dirty.append(key)
        i = self._chunk_of[key]
        marked = self._marked.setdefault(i, set())
        marked.add(key)
        if self.eager_launch and len(marked) == len(self._chunks[i][2]):
            self._launch_chunk(i, 'hook')
            done = set(self._chunks[i][2])
            self._dirty = [k for k in self._dirty if k not in done]

    def pending(self, key: Any) -> bool:
        return key in self._dirty

    def _launch_chunk(self, i: int, where: str) -> None:
        assert self.flat is not None
        start, end, keys = self._chunks[i]
        work = dist.all_reduce(self.flat[start:end], group=self.group, async_op=True)
        for k in keys:
            self._works[k] = work
        self._marked.pop(i, None)
        self.launch_log.append((i, where))

    def launch(self) -> None:
        """All-reduce every chunk still holding a marked slot (collective)."""
        if not self._dirty:
            return
        assert self.flat is not None
        todo = sorted({self._chunk_of[k] for k in self._dirty})
        self._dirty = []
        for i in todo:
            self._launch_chunk(i, 'step')
        self.launches += 1

    def wait(self, key: Any) -> None:
        """Order the current stream after the slot's last all-reduce."""
        w = self._works.pop(key, None)
        if w is not None:
            w.wait()


class _SlotHandle:
    """Bucket-like handle an ``AsyncTensor`` waits on for one packed slot."""

    __slots__ = ('_buf', '_key')

    def __init__(self, buf: PackedFactorBuffer, key: Any) -> None:
        self._buf = buf
        self._key = key

    def communicated(self) -> bool:
        return not self._buf.pending(self._key)

    @property
    def work(self) -> Any:
        return self._buf._works.pop(self._key, None)


class TorchDistributedCommunicator:
    """All-reduce / broadcast helper used by every K-FAC layer.

    Args:
        bucket_cap_mb (float): cap of a fused all-reduce bucket in decimal MB
            (1e6 bytes), as in the reference (``distributed.py:137-140``).
    """

    def __init__(self, bucket_cap_mb: float = 25.0) -> None:
        self._bucket_cap_mb = bucket_cap_mb
        self._bucket_cap_bytes = int(bucket_cap_mb * 1000 * 1000)
        self._allreduce_buckets: dict[Any, AllreduceTensorBucket | None] = {}
        self._broadcast_buckets: dict[Any, BroadcastTensorBucket] = {}
        self._exchange_buckets: dict[Any, ExchangeTensorBucket] = {}
        self._packed: dict[Any, PackedFactorBuffer] = {}

    def packed_buffer(self, group: dist.ProcessGroup | None, dtype: torch.dtype,
                      device: torch.device) -> PackedFactorBuffer:
        """The persistent packed-factor buffer of ``group``."""
        key = (group, dtype, str(device))
        buf = self._packed.get(key)
        if buf is None:
            buf = PackedFactorBuffer(group, self._bucket_cap_bytes)
            self._packed[key] = buf
        return buf

    def packed_result(self, buf: PackedFactorBuffer, key: Any,
                      finalize: Callable[[], torch.Tensor]) -> AsyncTensor:
        """Handle resolving to ``finalize()`` once the slot is reduced."""
        return AsyncTensor(finalize=finalize, bucket=_SlotHandle(buf, key))  # type: ignore[arg-type]

    @property
    def bucket_cap_bytes(self) -> int:
        return self._bucket_cap_bytes

    @property
    def bucket_cap_mb(self) -> float:
        return self._bucket_cap_mb

    def group_ranks(self, group: dist.ProcessGroup | None) -> frozenset[int]:
        """Global ranks of ``group`` (all ranks for the world group)."""
        if group is None or not dist.is_initialized():
            return frozenset(range(get_world_size(group)))
        return frozenset(dist.get_process_group_ranks(group))

    @staticmethod
    def _check_square(tensor: torch.Tensor) -> None:
        if tensor.dim() != 2 or tensor.shape[0] != tensor.shape[1]:
            raise NonSquareTensorError(
                'Symmetric communication can only be done with a 2D square '
                f'tensor. Got tensor with shape {tuple(tensor.shape)}.',
            )

    def allreduce(
        self,
        tensor: torch.Tensor,
        *,
        average: bool = False,
        group: dist.ProcessGroup | None = None,
        symmetric: bool = False,
    ) -> AsyncTensor | torch.Tensor:
        """Asynchronous (optionally averaged / triangle-packed) all-reduce.

        Returns ``tensor`` itself when the group has one rank.  Otherwise an
        ``AsyncTensor`` whose value is ``tensor`` updated in place.
        """
        if get_world_size(group) == 1:
            return tensor
        if symmetric:
            self._check_square(tensor)
        scale = _scale_for(average, group)
        if symmetric:
            wire = comm_pack.triu_pack(tensor)
        elif tensor.is_contiguous():
            wire = tensor
        else:
            wire = tensor.contiguous()
        work = dist.all_reduce(wire, group=group, async_op=True)
        target = _result_buffer(tensor, wire, symmetric)

        def _finish() -> torch.Tensor:
            if symmetric:
                comm_pack.triu_unpack_(target, wire, scale)
            elif scale != 1.0:
                target.mul_(scale)
            return target

        return AsyncTensor(work=work, finalize=_finish)

    def broadcast(
        self,
        tensor: torch.Tensor,
        *,
        src: int,
        group: dist.ProcessGroup | None = None,
        symmetric: bool = False,
    ) -> AsyncTensor | torch.Tensor:
        """Asynchronous broadcast from global rank ``src`` within ``group``."""
        if get_world_size(group) == 1:
            return tensor
        if symmetric:
            self._check_square(tensor)
            wire = comm_pack.triu_pack(tensor)
        else:
            wire = tensor if tensor.is_contiguous() else tensor.contiguous()
        work = dist.broadcast(wire, src=src, group=group, async_op=True)
        target = _result_buffer(tensor, wire, symmetric)

        def _finish() -> torch.Tensor:
            if symmetric:
                comm_pack.triu_unpack_(target, wire, 1.0)
            return target

        return AsyncTensor(work=work, finalize=_finish)

    def allreduce_bucketed(
        self,
        tensor: torch.Tensor,
        *,
        average: bool = False,
        group: dist.ProcessGroup | None = None,
        symmetric: bool = False,
    ) -> AsyncTensor | torch.Tensor:
        """All-reduce through a fused bucket (launched when full or flushed).

        A bucket never exceeds the cap unless it holds a single tensor larger
        than the cap.  The value written back in place into ``tensor``.
        """
        if get_world_size(group) == 1:
            return tensor
        if symmetric:
            self._check_square(tensor)
        scale = _scale_for(average, group)
        nbytes = comm_pack.packed_numel(tensor, symmetric) * tensor.element_size()
        key = group
        bucket = self._allreduce_buckets.get(key)
        if bucket is None:
            bucket = AllreduceTensorBucket(group)
            self._allreduce_buckets[key] = bucket
        elif bucket.size + nbytes > self._bucket_cap_bytes:
            bucket.allreduce()
            bucket = AllreduceTensorBucket(group)
            self._allreduce_buckets[key] = bucket

        target = tensor

        def _finish(sl: torch.Tensor) -> torch.Tensor:
            if not target.is_contiguous():
                raise RuntimeError('bucketed all-reduce needs contiguous tensors')
            comm_pack.unpack_slice_(target, sl, symmetric, scale)
            return target

        return bucket.add_tensor(tensor, symmetric=symmetric, finalize=_finish)

    def broadcast_bucketed(
        self,
        tensor: torch.Tensor,
        *,
        src: int,
        group: dist.ProcessGroup | None = None,
    ) -> AsyncTensor | torch.Tensor:
        """Broadcast through a flat bucket per (group, src).

        Used for the per-step preconditioned-gradient broadcasts:
        ResNet-50 would otherwise issue 54 small RCCL broadcasts per step.
        Buckets are launched when full (``bucket_cap_mb``) or on
        ``flush_broadcast_buckets()``; every rank of ``group`` must add the
        same tensors (shapes) in the same order.  The value is written in
        place into ``tensor`` on receivers.
        """
        if get_world_size(group) == 1:
            return tensor
        if not tensor.is_contiguous():
            raise RuntimeError('bucketed broadcast needs contiguous tensors')
        key = (group, src)
        nbytes = tensor.numel() * tensor.element_size()
        bucket = self._broadcast_buckets.get(key)
        if bucket is None:
            bucket = BroadcastTensorBucket(group, src)
            self._broadcast_buckets[key] = bucket
        elif bucket.size + nbytes > self._bucket_cap_bytes:
            bucket.broadcast()
            bucket = BroadcastTensorBucket(group, src)
            self._broadcast_buckets[key] = bucket
        return bucket.add_tensor(tensor)

    def exchange_bucketed(
        self,
        tensor: torch.Tensor,
        *,
        src: int,
        group: dist.ProcessGroup | None = None,
    ) -> AsyncTensor | torch.Tensor:
        """Broadcast ``tensor`` from ``src`` to ``group`` through a per-group
        exchange bucket: at flush every member contributes the tensors it is
        the source of and receives the others' in ONE all-gather.

        Used for the per-step preconditioned-gradient broadcasts (SURVEY C5:
        every member of a KAISA receiver group is the source of some layers).
        Per-(group, src) broadcasts run one after another on the group's
        communicator, each using the links in one direction; the all-gather
        sends every member's share at once, both directions of every xGMI
        link busy (2-rank groups: half the time).  Same values, bit for bit,
        as the broadcasts (``kfac/layers/base.py:223-251`` in the reference).
        Every rank of ``group`` must add the same tensors (shapes, sources) in
        the same order; the result is written in place on receivers."""
        if get_world_size(group) == 1:
            return tensor
        if not tensor.is_contiguous():
            raise RuntimeError('bucketed exchange needs contiguous tensors')
        key = group
        nbytes = tensor.numel() * tensor.element_size()
        bucket = self._exchange_buckets.get(key)
        if bucket is None:
            bucket = ExchangeTensorBucket(group)
            self._exchange_buckets[key] = bucket
        elif bucket.size + nbytes > self._bucket_cap_bytes * get_world_size(group) or (
                bucket.dtype is not None and bucket.dtype != tensor.dtype):
            bucket.exchange()
            bucket = ExchangeTensorBucket(group)
            self._exchange_buckets[key] = bucket
        return bucket.add_tensor(tensor, src)

    def flush_broadcast_buckets(self) -> None:
        """Launch every pending broadcast and exchange bucket, in creation
        order."""
        for key in list(self._broadcast_buckets):
            bucket = self._broadcast_buckets.pop(key)
            bucket.broadcast()
        for key in list(self._exchange_buckets):
            self._exchange_buckets.pop(key).exchange()

    def flush_allreduce_buckets(self) -> None:
        """Launch every partially filled bucket and every packed-factor
        buffer with marked slots (collective on all ranks)."""
        for key in list(self._allreduce_buckets):
            bucket = self._allreduce_buckets[key]
            if bucket is not None:
                bucket.allreduce()
                self._allreduce_buckets[key] = None
        for buf in self._packed.values():
            buf.launch()


class BroadcastTensorBucket:
    """A fused broadcast of several same-dtype tensors from one source."""

    def __init__(self, group: dist.ProcessGroup | None, src: int) -> None:
        self._group = group
        self._src = src
        self._tensors: list[torch.Tensor] = []
        self._size = 0
        self._sent = False
        self.work: Any | None = None
        self.flat: torch.Tensor | None = None

    @property
    def size(self) -> int:
        return self._size

    def communicated(self) -> bool:
        return self._sent

    def add_tensor(self, tensor: torch.Tensor) -> AsyncTensor:
        if self._sent:
            raise RuntimeError('bucket was already communicated')
        if self._tensors and tensor.dtype != self._tensors[0].dtype:
            raise RuntimeError('a broadcast bucket holds a single dtype')
        offset = sum(t.numel() for t in self._tensors)
        n = tensor.numel()
        self._tensors.append(tensor)
        self._size += n * tensor.element_size()
        is_src = get_rank() == self._src

        def _finish() -> torch.Tensor:
            assert self.flat is not None
            sl = self.flat[offset: offset + n]
            if not is_src and sl.data_ptr() != tensor.data_ptr():
                comm_pack.scale_copy_(tensor, sl, 1.0)
            return tensor

        return AsyncTensor(finalize=_finish, bucket=self)  # type: ignore[arg-type]

    def allreduce(self) -> Any:  # AsyncTensor resolves through .work
        return self.broadcast()

    def broadcast(self) -> Any | None:
        if self._sent:
            raise RuntimeError('bucket was already communicated')
        self._sent = True
        if not self._tensors:
            return None
        ref = self._tensors[0]
        total = sum(t.numel() for t in self._tensors)
        if len(self._tensors) == 1:
            self.flat = ref.view(-1)
        else:
            self.flat = torch.empty(total, dtype=ref.dtype, device=ref.device)
            if get_rank() == self._src:
                off = 0
                for t in self._tensors:
                    self.flat[off: off + t.numel()].copy_(t.view(-1))
                    off += t.numel()
        self.work = dist.broadcast(self.flat, src=self._src, group=self._group, async_op=True)
        return self.work


class ExchangeTensorBucket:
    """Tensors of one KAISA receiver group, each from one source member,
    exchanged by a single all-gather (``exchange_bucketed``).

    Every member packs the tensors it is the source of into a send buffer
    padded to the largest member's share; ``all_gather_into_tensor`` lays
    the shares out in group-rank order; receivers copy theirs out.  Sizes
    and sources are identical on every member, so every member computes the
    same layout without communicating it."""

    def __init__(self, group: dist.ProcessGroup | None) -> None:
        self._group = group
        self._entries: list[tuple[torch.Tensor, int, int]] = []  # tensor, src slot, offset
        self._fill: dict[int, int] = {}  # src slot -> numel so far
        self._size = 0
        self._sent = False
        self.dtype: torch.dtype | None = None
        self.work: Any | None = None
        self.flat: torch.Tensor | None = None
        self._pad = 0
        self._me = _group_rank(group, get_rank())

    @property
    def size(self) -> int:
        return self._size

    def communicated(self) -> bool:
        return self._sent

    def add_tensor(self, tensor: torch.Tensor, src: int) -> AsyncTensor:
        if self._sent:
            raise RuntimeError('bucket was already communicated')
        if self.dtype is not None and tensor.dtype != self.dtype:
            raise RuntimeError('an exchange bucket holds a single dtype')
        self.dtype = tensor.dtype
        slot = _group_rank(self._group, src)
        off = self._fill.get(slot, 0)
        n = tensor.numel()
        self._fill[slot] = off + n
        self._entries.append((tensor, slot, off))
        self._size += n * tensor.element_size()

        def _finish() -> torch.Tensor:
            if slot != self._me:
                assert self.flat is not None
                start = slot * self._pad + off
                comm_pack.scale_copy_(tensor, self.flat[start: start + n], 1.0)
            return tensor

        return AsyncTensor(finalize=_finish, bucket=self)  # type: ignore[arg-type]

    def allreduce(self) -> Any:  # AsyncTensor resolves through .work
        return self.exchange()

    def exchange(self) -> Any | None:
        if self._sent:
            raise RuntimeError('bucket was already communicated')
        self._sent = True
        if not self._entries:
            return None
        size = get_world_size(self._group)
        self._pad = max(self._fill.values())
        ref = self._entries[0][0]
        send = torch.zeros(self._pad, dtype=ref.dtype, device=ref.device)
        for t, slot, off in self._entries:
            if slot == self._me:
                send[off: off + t.numel()].copy_(t.view(-1))
        self.flat = torch.empty(size * self._pad, dtype=ref.dtype, device=ref.device)
        self.work = dist.all_gather_into_tensor(self.flat, send, group=self._group,
                                                async_op=True)
        return self.work


def _group_rank(group: dist.ProcessGroup | None, global_rank: int) -> int:
    """Rank of ``global_rank`` inside ``group`` (its position in an
    all-gather's output)."""
    if group is None or not (dist.is_available() and dist.is_initialized()):
        return global_rank
    return dist.get_group_rank(group, global_rank)
