"""Multi-process pair sharding (scatter -> per-rank forward -> gather) on the gloo backend, CPU tensors,
world_size 2 and 3 — the same code path bench.py runs over RCCL on GPUs."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from model.pair_sharding import gather_flows, infer_sharded, scatter_pairs, shard_bounds


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_forward(a, b):
    # stands in for RAFT: any per-pair function; flow_low from pooled difference, flow_up full res
    low = torch.nn.functional.avg_pool2d(b[:, :2] - a[:, :2], 8)
    return low, (a[:, :2] * 0.5 + b[:, 1:3])


def _worker(rank, world, port, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        img0 = torch.rand(batch, 3, 16, 24, generator=g) * 255
        img1 = torch.rand(batch, 3, 16, 24, generator=g) * 255
        s0, s1 = scatter_pairs(img0 if rank == 0 else None, img1 if rank == 0 else None, torch.device("cpu"))
        st, sp = shard_bounds(batch, world, rank)
        ok_scatter = torch.equal(s0, img0[st:sp]) and torch.equal(s1, img1[st:sp])
        back = gather_flows(s0[:, :2].contiguous(), batch)
        ok_gather = (back is None) if rank else torch.equal(back, img0[:, :2])
        low, up = infer_sharded(_fake_forward, img0 if rank == 0 else None, img1 if rank == 0 else None, torch.device("cpu"))
        if rank == 0:
            rl, ru = _fake_forward(img0, img1)
            ok_inf = torch.equal(low, rl) and torch.equal(up, ru)
        else:
            ok_inf = low is None and up is None
        q.put((rank, ok_scatter, ok_gather, ok_inf))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 8), (2, 5), (3, 7)])
def test_scatter_gather_gloo(world, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(all(r[1:]) for r in res), res


def test_shard_bounds_cover_batch():
    for b in range(0, 20):
        for w in range(1, 9):
            spans = [shard_bounds(b, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == b
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(s1 - s0 for s0, s1 in spans) - min(s1 - s0 for s0, s1 in spans) <= 1
