"""World-size-2 gloo tests of the sample-sharded multi-GPU logic (CPU, no GPU needed):
shard partition, weight broadcast (C1), gather (C2) and shard-invariant host noise."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dmx import distributed as dd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_shard_range_partitions():
    for total in (1, 7, 64, 512, 513):
        for ws in (1, 2, 3, 8):
            spans = [dd.shard_range(total, ws, r) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def _bcast_gather(rank, world):
    m = torch.nn.Linear(4, 3)
    if rank == 0:
        with torch.no_grad():
            m.weight.fill_(1.5)
            m.bias.fill_(-2.0)
    dd.broadcast_module(m)
    local = torch.arange(dd.shard_range(5, world, rank)[0], dd.shard_range(5, world, rank)[1]).float().unsqueeze(1)
    full = dd.gather_rows(local, 5)
    return float(m.weight.sum()), float(m.bias.sum()), None if full is None else full.flatten().tolist()


def test_broadcast_and_gather_world2():
    res = run(_bcast_gather)
    for r in (0, 1):
        assert res[r][0] == 1.5 * 12 and res[r][1] == -6.0
    assert res[0][2] == [0.0, 1.0, 2.0, 3.0, 4.0] and res[1][2] is None


def _toy_step(x, t, noise):
    return 0.9 * x + 0.05 * t * 1e-3 + 0.1 * noise


def _sharded_host_noise(rank, world):
    torch.manual_seed(123)
    x = dd.sharded_loop(_toy_step, (5, 2, 3, 3), 6, "cpu", "host")
    return dd.gather_rows(x, 5)


def test_host_noise_is_shard_invariant_world2():
    """Each sample's x_T and per-step noise equal the single-process draw order (diff.py:327,158)."""
    res = run(_sharded_host_noise)
    torch.manual_seed(123)
    x = torch.randn((5, 2, 3, 3))
    for i in range(6, 0, -1):
        x = _toy_step(x, i, torch.randn((5, 2, 3, 3)))
    assert torch.equal(res[0], x)
