"""CPU, world_size 2/4/8 over gloo: the N>1 sharding contract (ranges, keyed noise slicing, final gather)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from weatherconverter_amd.diffusion_model.distributed import gather_samples, shard_range


def test_shard_range_partitions():
    for total in (1, 7, 16, 128, 129):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == total
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, total, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        start, count = shard_range(total, world, rank)
        # per-sample keyed "trajectory": each rank computes only its rows from the global index
        rows = torch.arange(start, start + count, dtype=torch.float32)
        x_local = rows[:, None, None, None].expand(count, 3, 4, 4) * 1.5 + torch.arange(48.).reshape(1, 3, 4, 4)
        # reference-RNG mode: every rank draws the FULL-batch tensor and keeps its rows
        torch.manual_seed(1234)
        full_noise = torch.randn((total, 3, 4, 4))
        x_local = x_local + full_noise[start:start + count]
        out = gather_samples(x_local.contiguous(), total)
        # by value: a shared-memory tensor handle can outlive this worker's fd sharer
        q.put((rank, out.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,total', [(2, 4), (2, 5), (4, 7), (8, 5)])
def test_gloo_gather_equals_single_rank(world, total):
    """world 8 with 5 samples leaves three ranks with an empty shard (the rehearsal of the driver's N=8 run)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: torch.from_numpy(a) for r, a in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(1234)
    noise = torch.randn((total, 3, 4, 4))
    ref = torch.arange(total, dtype=torch.float32)[:, None, None, None] * 1.5 + torch.arange(48.).reshape(1, 3, 4,
                                                                                                          4) + noise
    for r in range(world):
        assert torch.equal(res[r], ref)
