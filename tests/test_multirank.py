"""The N>1 path of bench.py on CPU: gloo ranks, as torch.distributed.run launches them.

Each rank takes its interleaved slice of ONE frame's film-pixel tiles (pbrtgpu.tile_slice,
the dealing of pbrtgpu_render_multi), renders a film and writes its slice's pixels into the
shared host film (bench.shared_film) -- the host gather of SURVEY.md §8(e), no collective on
the data path.  Here the per-rank renderer is the CPU oracle (no GPU in this container); the
gathered film must equal the oracle's full-frame film bit for bit, the slices must partition
the tiles, and the timing reduction is the max over ranks (paths summed)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, PACKS


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def tile_mask(pg, scene, tiles, tile=16):
    """Film pixels of a tile list (the grid of pbrtgpu.h / tile_pixels in pbrtgpu.hip)."""
    m = np.zeros((scene.height, scene.width), bool)
    ntx, _ = pg.tile_grid(scene, tile)
    for t in tiles:
        ty, tx = divmod(int(t), ntx)
        m[ty * tile:(ty + 1) * tile, tx * tile:(tx + 1) * tile] = True
    return m


def _worker(rank, world, port, q, mode="shared"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
    import bench
    import pbrtgpu as pg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"), xres=40, yres=36, spp=2)
    ntx, nty = pg.tile_grid(scene)
    tiles = pg.tile_slice(ntx * nty, rank, world)
    shape = (scene.height, scene.width, scene.bands)
    if mode == "shared":   # all ranks on one node: the /dev/shm film
        path, film = bench.shared_film(shape, rank, dist, "test_%d" % port)
    else:                  # ranks on several nodes: private films, summed onto rank 0 afterwards
        path, film = None, np.zeros(shape, np.float32)
    mine, _ = pg.oracle().render(scene, threads=2)       # this rank's film (stands in for its GPU)
    m = tile_mask(pg, scene, tiles)
    film[m] = mine[m]                                    # host gather of the slice's pixels
    if mode == "shared":
        film.flush()
    else:
        film = bench.compose_film(film, dist)
    elapsed, total = bench.reduce_over_ranks(dist, 1.0 + rank, 100.0 * (rank + 1))
    dist.barrier()
    if rank == 0:
        full, _ = pg.oracle().render(scene, threads=2)
        same = bool(np.array_equal(np.asarray(film).view(np.int32), full.view(np.int32)))
        if path:
            os.unlink(path)
    else:
        same = None
    q.put((rank, tiles.tolist(), int(ntx * nty), elapsed, total, same))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "shared"), (3, "shared"), (2, "compose")])
def test_tile_slices_gather_and_reduction(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ntiles = res[0][2]
    tiles = sorted(t for _, ts, _, _, _, _ in res for t in ts)
    assert tiles == list(range(ntiles))
    for _, ts, _, elapsed, total, _ in res:
        assert abs(len(ts) - ntiles / world) <= 1
        assert elapsed == float(world) and total == 100.0 * world * (world + 1) / 2
    assert res[0][5] is True


def test_tile_slices_match_render_multi_dealing(pg):
    """tile_slice(n, j, m) is slice j of pbrtgpu_render_multi's dealing: list[j::m]."""
    for n, m in [(1936, 8), (16, 3), (5, 8)]:
        got = np.concatenate([pg.tile_slice(n, j, m) for j in range(m)])
        assert sorted(got.tolist()) == list(range(n))
        for j in range(m):
            assert pg.tile_slice(n, j, m).tolist() == list(range(n))[j::m]


def test_one_node_detection(monkeypatch):
    """bench.py uses the /dev/shm film only when every rank is on this node (torchrun's
    LOCAL_WORLD_SIZE == WORLD_SIZE); otherwise each rank keeps its own film (compose_film)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert bench.one_node(8) and not bench.one_node(16)
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    assert bench.one_node(4)
