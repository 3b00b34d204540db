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


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,batch", [(2, 8), (2, 5), (3, 7), (3, 2)])
def test_scatter_gather_gloo(world, batch):
    """Includes batch < world (rank 2 of (3, 2) holds no pair: it skips the forward and pads the gather)."""
    res = _run(_worker, world, batch)
    assert all(all(r[1:]) for r in res), res


def _oracle_worker(rank, world, port, batch, known_shape, q):
    """The oracle RAFT (PyTorch-CPU restatement of the reference) sharded over gloo vs the same model unsharded."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from model import synthetic
        from oracle import raft as oraft

        model = oraft.RAFT().eval()
        model.load_state_dict(synthetic.synthetic_state_dict(model.state_dict()))
        h, w = 128, 128  # level 3 = 2x2 (a 1-px level is NaN in the reference, Q3)
        img0, img1 = synthetic.synthetic_pair(batch, h, w, seed=4)

        def forward(a, b):
            return model(a, b, iters=3, test_mode=True)

        with torch.inference_mode():
            shape = (batch, 3, h, w) if known_shape else None
            flows = ((2, h // 8, w // 8), (2, h, w)) if known_shape else None
            low, up = infer_sharded(forward, img0 if rank == 0 else None, img1 if rank == 0 else None,
                                    torch.device("cpu"), shape=shape, flow_shapes=flows)
            if rank == 0:
                rl, ru = forward(img0, img1)
                d = max(float((low - rl).abs().max()), float((up - ru).abs().max()))
                q.put((rank, d, tuple(up.shape)))
            else:
                q.put((rank, 0.0 if low is None and up is None else 1.0, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch,known_shape", [(2, 3, True), (2, 2, False), (3, 2, True)])
def test_oracle_raft_sharded_equals_unsharded(world, batch, known_shape):
    """sharding pairs over ranks is exact -- each pair's flow from its rank equals the unsharded batch
    run of the same model (per-pair math; the CPU convolutions are batch-size invariant to <= 1e-5 px)."""
    res = sorted(_run(_oracle_worker, world, batch, known_shape))
    assert res[0][2] == (batch, 2, 128, 128)
    assert res[0][1] <= 1e-5, res
    assert all(r[1] == 0.0 for r in res[1:]), res


def test_shard_bounds_cover_batch():
    for b in range(0, 20):
        for w in range(1, 9):
            spans = [shard_bounds(b, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == b
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(s1 - s0 for s0, s1 in spans) - min(s1 - s0 for s0, s1 in spans) <= 1


def _shape_worker(rank, world, port, q):
    """Rank 0 holds 3 pairs but every rank is told (4, 3, 16, 24): the one-time collective check raises on every
    rank. Then, after a step with the right shape, rank 0's batch changes: rank 0 raises after completing the
    collectives with NaN pieces; the peers return (NaN shard / no flows) instead of blocking."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        src_img = torch.zeros(3, 3, 16, 24) if rank == 0 else None
        try:
            scatter_pairs(src_img, src_img, torch.device("cpu"), shape=(4, 3, 16, 24))
            out.append("no-error")
        except ValueError:
            out.append("ValueError")
        good = torch.ones(4, 3, 16, 24) if rank == 0 else None
        s0, _ = scatter_pairs(good, good, torch.device("cpu"), shape=(4, 3, 16, 24))
        out.append("ok" if bool((s0 == 1).all()) else "bad")
        bad = torch.ones(5, 3, 16, 24) if rank == 0 else None  # changed after the check
        try:
            s0, _ = scatter_pairs(bad, bad, torch.device("cpu"), shape=(4, 3, 16, 24))
            out.append("nan" if bool(torch.isnan(s0).all()) else "values")
        except ValueError:
            out.append("ValueError")
        try:
            low, up = infer_sharded(_fake_forward, bad, bad, torch.device("cpu"), shape=(4, 3, 16, 24),
                                    flow_shapes=((2, 2, 3), (2, 16, 24)))
            out.append("none" if low is None and up is None else "flows")
        except ValueError:
            out.append("ValueError")
        q.put((rank, tuple(out)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_scatter_refuses_a_shape_that_disagrees_with_the_batch(world):
    """A caller-given global shape that disagrees with the source batch fails on every rank (one-time collective
    check), and a later change of the source batch fails on the source without leaving a peer blocked in a
    collective (the test's queue timeout would catch a hang)."""
    res = sorted(_run(_shape_worker, world))
    assert res[0] == (0, ("ValueError", "ok", "ValueError", "ValueError"))
    for r in res[1:]:
        assert r[1] == ("ValueError", "ok", "nan", "none"), r


def _pipeline_worker(rank, world, port, batch, steps, reuse, q):
    """infer_sharded_pipelined (scatter of step i+1 and gathers of step i in flight around step i's forward) vs
    infer_sharded step by step, on distinct batches per step. ``reuse``: the forward returns the same two output
    buffers every call, overwritten in place (as GraphedRAFT's replayed outputs are)."""
    from model.pair_sharding import infer_sharded_pipelined

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(1)
        data = [(torch.rand(batch, 3, 16, 24, generator=g) * 255, torch.rand(batch, 3, 16, 24, generator=g) * 255)
                for _ in range(steps)]
        cpu = torch.device("cpu")
        shape = (batch, 3, 16, 24)
        flow_shapes = ((2, 2, 3), (2, 16, 24))
        seq = [infer_sharded(_fake_forward, *(d if rank == 0 else (None, None)), cpu, shape=shape, flow_shapes=flow_shapes)
               for d in data]
        calls = []
        bufs = {}

        def fwd(a, b):
            calls.append(a.shape[0])
            lo, up = _fake_forward(a, b)
            if not reuse:
                return lo, up
            if not bufs:
                bufs["lo"], bufs["up"] = torch.empty_like(lo), torch.empty_like(up)
            bufs["lo"].copy_(lo)
            bufs["up"].copy_(up)
            return bufs["lo"], bufs["up"]

        batches = (d if rank == 0 else (None, None) for d in data)
        pipe = list(infer_sharded_pipelined(fwd, batches, cpu, shape=shape, flow_shapes=flow_shapes))
        ok = len(pipe) == steps
        for (lo, up), (rl, ru) in zip(pipe, seq):
            if rank == 0:
                ok = ok and torch.equal(lo, rl) and torch.equal(up, ru)
            else:
                ok = ok and lo is None and up is None and rl is None and ru is None
        st, sp = shard_bounds(batch, world, rank)
        ok = ok and calls == ([sp - st] * steps if sp > st else [])
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch,steps,reuse", [(2, 8, 3, False), (2, 5, 1, False), (3, 2, 2, False),
                                                     (2, 8, 4, True), (3, 7, 3, True)])
def test_pipelined_steps_equal_sequential_gloo(world, batch, steps, reuse):
    """The overlapped step driver bench.py --gpus N uses returns every step's flows exactly as the sequential
    scatter -> forward -> gather does, including a ragged batch, one step, a rank without pairs, and a forward that
    overwrites one pair of output buffers per call (the gathers still in flight send private copies)."""
    res = _run(_pipeline_worker, world, batch, steps, reuse)
    assert all(r[1] for r in res), res
