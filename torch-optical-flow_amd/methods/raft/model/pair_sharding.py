"""Image-pair batch sharding over one process per GPU (``torch.distributed``; backend "nccl" = RCCL on ROCm).

Every image pair is an independent RAFT forward (no cross-pair state; cnet BatchNorm uses running statistics
in eval mode), so the only communication is at the edges of the batch:
  * ``scatter_pairs``: rank ``src`` holds the global (B, 3, H, W) pair batch and scatters contiguous shards,
    one per rank (RCCL lowers scatter to per-peer sends: each peer receives over its own xGMI link);
  * ``gather_flows``:  shards' flows go back to rank ``dst``.
There is no per-iteration exchange, and with the global shape passed in (fixed per run; checked against the source
batch once, collectively) a step issues only the scatter and the two gathers: no metadata broadcast, no host sync. Ragged batches (B % world_size != 0) are padded
to equal chunks for the collective and trimmed on both sides; a rank with no pair skips the forward. The same code runs on gloo with CPU tensors (tests).
"""
from __future__ import annotations

from typing import Callable, Iterable, Iterator, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor


def shard_bounds(global_batch: int, world_size: int, rank: int) -> Tuple[int, int]:
    """[start, stop) of ``rank``'s contiguous shard; shards differ in size by at most one pair."""
    base, extra = divmod(global_batch, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _world(group) -> Tuple[int, int]:
    return dist.get_world_size(group), dist.get_rank(group)


def _meta(t: Optional[Tensor], src: int, group, device: torch.device) -> Sequence[int]:
    """Broadcast ``t``'s shape from ``src`` (only when the caller does not pass it: one small collective + one host
    sync). The rank count travels first, so zero-sized dimensions survive."""
    rank = dist.get_rank(group)
    meta = torch.zeros(9, dtype=torch.int64, device=device)
    if rank == src:
        meta[0] = t.dim()
        meta[1 : 1 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
    dist.broadcast(meta, src=dist.get_global_rank(group, src) if group is not None else src, group=group)
    v = meta.tolist()
    return v[1 : 1 + v[0]]


_VALIDATED = set()  # (shape, process group object, world size, src) checked collectively (see scatter_pairs)


def _group_key(group):
    """The process group itself (the key holds a reference, so a destroyed and re-created group -- a new object -- is
    validated again) with its size."""
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    return pg, dist.get_world_size(group)


def _check_shape_collectively(shape, image0, image1, src: int, group, device: torch.device) -> None:
    """Once per (shape, group, src) per process: rank ``src`` broadcasts whether its batch matches the caller-given
    global ``shape`` and every rank raises the same ValueError on a mismatch (one 8-byte broadcast + one host sync
    per run, not per step)."""
    world, rank = _world(group)
    key = (tuple(int(v) for v in shape), *_group_key(group), src)
    if key in _VALIDATED:
        return
    ok = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == src:
        ok[0] = int(all(tuple(img.shape) == tuple(shape) for img in (image0, image1)))
    dist.broadcast(ok, src=dist.get_global_rank(group, src) if group is not None else src, group=group)
    if not int(ok.item()):
        got = tuple(image0.shape) if rank == src else "(held by the source rank)"
        raise ValueError(f"scatter_pairs: shape {tuple(shape)} does not match the source batch {got}")
    _VALIDATED.add(key)


def _src_rank(group, src):
    return dist.get_global_rank(group, src) if group is not None else src


def _scatter(image0, image1, device, src, group, shape, async_op: bool = False):
    """The scatter; returns (shard0, shard1, error). A source batch that disagrees with a caller-given ``shape`` after
    the one-time collective check (the source's batch changed shape mid-run) still completes the collective with
    NaN pieces of the agreed size, so no peer blocks; the source gets the ValueError back to raise afterwards."""
    world, rank = _world(group)
    err = None
    if shape is not None:
        _check_shape_collectively(shape, image0, image1, src, group, device)
        if rank == src and any(tuple(img.shape) != tuple(shape) for img in (image0, image1)):
            err = ValueError(f"scatter_pairs: shape {tuple(shape)} does not match the source batch {tuple(image0.shape)}")
    shape = list(shape) if shape is not None else _meta(image0, src, group, device)
    b, rest = shape[0], shape[1:]
    chunk = -(-b // world)
    start, stop = shard_bounds(b, world, rank)
    outs, works = [], []
    for img in (image0, image1):
        recv = torch.empty([chunk] + rest, dtype=torch.float32, device=device)
        scatter_list = None
        if rank == src:
            scatter_list = []
            if err is not None:  # poison: the agreed sizes, NaN values
                scatter_list = [torch.full([chunk] + rest, float("nan"), device=device) for _ in range(world)]
            else:
                img = img.to(device=device, dtype=torch.float32)
                for r in range(world):
                    s0, s1 = shard_bounds(b, world, r)
                    piece = img[s0:s1]
                    if s1 - s0 < chunk:
                        piece = torch.cat([piece, piece.new_zeros([chunk - (s1 - s0)] + rest)], dim=0)
                    scatter_list.append(piece.contiguous())
        w = dist.scatter(recv, scatter_list, src=_src_rank(group, src), group=group, async_op=async_op)
        works.append(w)
        outs.append(recv[: stop - start])
    if async_op:
        return outs[0], outs[1], err, works
    return outs[0], outs[1], err


def scatter_pairs(
    image0: Optional[Tensor],
    image1: Optional[Tensor],
    device: torch.device,
    src: int = 0,
    group=None,
    shape: Optional[Sequence[int]] = None,
) -> Tuple[Tensor, Tensor]:
    """Scatter the pair batch held by rank ``src`` (other ranks pass ``None``); returns this rank's shard.
    ``shape`` = the global (B, C, H, W) when every rank knows it (fixed per run: after a one-time collective check that
    it matches the source batch -- a mismatch raises ValueError on every rank -- a step issues no metadata collective
    and no host sync); otherwise it is broadcast from ``src``. Should the source batch later stop matching ``shape``,
    the source raises ValueError after completing the collective with NaN pieces (peers receive NaN, never block)."""
    s0, s1, err = _scatter(image0, image1, device, src, group, shape)
    if err is not None:
        raise err
    return s0, s1


class _PendingGather:
    """An issued (async) gather of flow shards to ``dst``: ``result()`` waits for it and returns the (B, ...) batch on
    ``dst``, None elsewhere."""

    __slots__ = ("work", "send", "gather_list", "global_batch", "world", "is_dst")

    def __init__(self, work, send, gather_list, global_batch: int, world: int, is_dst: bool) -> None:
        self.work, self.send, self.gather_list = work, send, gather_list
        self.global_batch, self.world, self.is_dst = global_batch, world, is_dst

    def result(self) -> Optional[Tensor]:
        if self.work is not None:
            self.work.wait()  # RCCL: the current stream waits for the collective (no host block); gloo: the host waits
        if not self.is_dst:
            return None
        parts = []
        for r in range(self.world):
            s0, s1 = shard_bounds(self.global_batch, self.world, r)
            parts.append(self.gather_list[r][: s1 - s0])
        return torch.cat(parts, dim=0)


def _gather(flow: Tensor, global_batch: int, dst: int, group, async_op: bool, own: bool = False) -> _PendingGather:
    """Issue the gather of ``flow`` (padded to the common chunk). ``own``: send a private copy even when ``flow`` is
    already a contiguous chunk, so that the caller may overwrite ``flow`` (a graph replay's output buffer, a reused
    workspace) while the gather is still reading on the communicator's stream; the copy is made on the current stream
    before the collective is issued, so it is ordered before the send."""
    world, rank = _world(group)
    chunk = -(-global_batch // world)
    rest = list(flow.shape[1:])
    if flow.shape[0] < chunk:
        send = torch.cat([flow, flow.new_zeros([chunk - flow.shape[0]] + rest)], dim=0)
    else:
        send = flow.clone(memory_format=torch.contiguous_format) if own else flow.contiguous()
    gather_list = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    w = dist.gather(send, gather_list, dst=_src_rank(group, dst), group=group, async_op=async_op)
    return _PendingGather(w, send, gather_list, global_batch, world, rank == dst)


def gather_flows(flow: Tensor, global_batch: int, dst: int = 0, group=None) -> Optional[Tensor]:
    """Gather every rank's (b_r, ...) flow shard to rank ``dst``; returns the (B, ...) batch there, else None."""
    return _gather(flow, global_batch, dst, group, async_op=False).result()


def infer_sharded(
    forward: Callable[[Tensor, Tensor], Tuple[Tensor, Tensor]],
    image0: Optional[Tensor],
    image1: Optional[Tensor],
    device: torch.device,
    src: int = 0,
    group=None,
    shape: Optional[Sequence[int]] = None,
    flow_shapes: Optional[Tuple[Sequence[int], Sequence[int]]] = None,
) -> Tuple[Optional[Tensor], Optional[Tensor]]:
    """scatter -> ``forward(shard0, shard1) -> (flow_low, flow_up)`` on every rank -> gather to ``src``.

    ``shape`` (global (B, C, H, W)) known on every rank makes a step collective-only: no metadata broadcast, no host
    sync (bench.py passes it; shapes are fixed per run). A rank whose shard is empty (B < world size) does not run
    ``forward``; it sends zero padding of ``flow_shapes`` = ((C, h, w) of flow_low, (C, H, W) of flow_up) -- without
    them it runs ``forward`` on one zero pair to learn the shapes and discards the result."""
    s0, s1, err = _scatter(image0, image1, device, src, group, shape)
    b = int(shape[0]) if shape is not None else None
    if b is None:
        gb = torch.tensor([image0.shape[0] if dist.get_rank(group) == src else 0], dtype=torch.int64, device=device)
        dist.broadcast(gb, src=dist.get_global_rank(group, src) if group is not None else src, group=group)
        b = int(gb.item())
    if s0.shape[0] == 0 or err is not None:  # no pair here, or a poisoned step on the source: pad the gathers
        if flow_shapes is None:
            z = s0.new_zeros([1] + list(s0.shape[1:]))
            lo, up = forward(z, z)
            flow_shapes = (lo.shape[1:], up.shape[1:])
        low = s0.new_zeros([0] + list(flow_shapes[0]))
        up = s0.new_zeros([0] + list(flow_shapes[1]))
    else:
        low, up = forward(s0, s1)
    out = gather_flows(low, b, dst=src, group=group), gather_flows(up, b, dst=src, group=group)
    if err is not None:  # every rank has completed the step's collectives
        raise err
    return out


def infer_sharded_pipelined(
    forward: Callable[[Tensor, Tensor], Tuple[Tensor, Tensor]],
    batches: Iterable[Tuple[Optional[Tensor], Optional[Tensor]]],
    device: torch.device,
    shape: Sequence[int],
    flow_shapes: Tuple[Sequence[int], Sequence[int]],
    src: int = 0,
    group=None,
) -> Iterator[Tuple[Optional[Tensor], Optional[Tensor]]]:
    """``infer_sharded`` over a stream of pair batches (rank ``src`` yields its (image0, image1) per step, the other
    ranks yield (None, None) the same number of times) with the communication off the compute stream's critical path:
    the scatter of step i+1 is issued (async) before step i's forward, so it runs on the RCCL stream while the forward
    runs, and step i's two gathers are issued right after its forward and overlap step i+1's forward. The compute stream
    waits for a step's scatter only when that step's forward starts (``work.wait()``: a stream-side wait under RCCL).
    Yields each step's (flow_low, flow_up) on ``src`` ((None, None) elsewhere) one step late, then the last one: the
    same flows, in the same order, as ``infer_sharded`` per step (tests/test_sharding_gloo.py). Collectives are issued
    in the same order on every rank: scatter 0, then per step i: scatter i+1, gathers i. Shapes are fixed for the run
    (``shape`` global (B, C, H, W), ``flow_shapes`` as in ``infer_sharded``).

    ``forward`` may return buffers it reuses on the next call (``GraphedRAFT``'s outputs are the graph's own and are
    overwritten by every replay): step i's gathers send private copies made on the compute stream before they are
    issued, so forward(i+1) cannot overwrite what the still-running gathers of step i read."""
    b = int(shape[0])
    it = iter(batches)

    def scatter(batch):
        s0, s1, err, works = _scatter(batch[0], batch[1], device, src, group, shape, async_op=True)
        return s0, s1, err, works

    cur = next(it, None)
    pend_scatter = scatter(cur) if cur is not None else None
    prev = None  # (gather low, gather up, err) of the previous step
    while pend_scatter is not None:
        s0, s1, err, works = pend_scatter
        for w in works:
            if w is not None:
                w.wait()
        nxt = next(it, None)
        pend_scatter = scatter(nxt) if nxt is not None else None  # in flight during this step's forward
        if s0.shape[0] == 0 or err is not None:
            low = s0.new_zeros([0] + list(flow_shapes[0]))
            up = s0.new_zeros([0] + list(flow_shapes[1]))
        else:
            low, up = forward(s0, s1)
        gathers = (_gather(low, b, src, group, async_op=True, own=True),
                   _gather(up, b, src, group, async_op=True, own=True), err)
        if prev is not None:
            out = prev[0].result(), prev[1].result()
            if prev[2] is not None:
                raise prev[2]
            yield out
        prev = gathers
    if prev is not None:
        out = prev[0].result(), prev[1].result()
        if prev[2] is not None:
            raise prev[2]
        yield out
