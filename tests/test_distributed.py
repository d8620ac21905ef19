"""Multi-process (world_size 2, gloo, CPU) tests of the batch sharding and the disparity
gather -- the only collective of the multi-GPU path."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from realtime_stereo_matcher_amd.distributed import gather_disparities, shard, shard_range


def test_shard_range_partitions():
    for gb in (0, 1, 7, 32):
        for world in (1, 2, 3, 8):
            spans = [shard_range(gb, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, global_batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.arange(global_batch * 2 * 3, dtype=torch.float32).view(global_batch, 1, 2, 3)
    mine = shard(full, rank, world) * 1.0  # stand-in for the per-rank regression output
    got = gather_disparities(mine.contiguous(), global_batch)
    if rank == 0:
        q.put(bool(torch.equal(got, full)))
    else:
        q.put(got is None)
    dist.destroy_process_group()


@pytest.mark.parametrize("global_batch", [4, 5])
def test_gather_world2_gloo(global_batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, global_batch, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    assert all(q.get(timeout=10) for _ in range(2))
