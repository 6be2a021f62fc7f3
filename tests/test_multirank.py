"""The N>1 path of bench.py on CPU: two gloo ranks, as torch.distributed.run launches them.
Tile sharding must partition a frame's tiles exactly; timing is the max over ranks and
paths are summed -- the only collectives (the path tracer itself exchanges nothing)."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ntiles, q):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tiles = bench.shard_tiles(ntiles, rank, world)
    elapsed, total = bench.reduce_over_ranks(dist, 1.0 + rank, 100.0 * (rank + 1), "cpu")
    q.put((rank, tiles.tolist(), elapsed, total))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tile_sharding_and_reduction():
    world, ntiles = 2, 1936   # 700x700 frame (+border) in 16x16 tiles
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, ntiles, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    tiles = sorted(t for _, ts, _, _ in res for t in ts)
    assert tiles == list(range(ntiles))
    for _, ts, elapsed, total in res:
        assert abs(len(ts) - ntiles / world) <= 1
        assert elapsed == 2.0 and total == 300.0
