"""GPU frame orchestration: how one frame is cut into pieces must never change its film.

- spp batches: a tiny per-sample radiance budget (PBRTGPU_LBUF_MB) forces many batches per
  frame, a tiny slot pool many wavefront runs per batch (the per-run drain bound);
- sample ranges: a frame rendered as [0, spp/2) + [spp/2, spp) with F_ACCUMULATE adds the same
  contributions, including exact-boundary samples, in a different float order;
- tiles: film-pixel tiles (pbrtgpu.h) at a resolution that is a multiple of the tile size;
- several contexts (pbrtgpu_render_multi, as for 8 GPUs; here two contexts on one GPU) and the
  host gather (pbrtgpu_film_gather);
- serial mode (PBRTGPU_SERIAL, the exclusive-timing mode of bench.py's roofline).

Reference semantics: SamplerRenderer::Render / SamplerRendererTask::Run
(renderers/samplerrenderer.cpp:60-222) with ComputeSubWindow task windows
(core/sampler.cpp:47-67) and SpectralImageFilm::AddSample (film/spectralImage.cpp:77-152).
"""
import os

import numpy as np
import pytest

from conftest import PACKS

pytestmark = pytest.mark.gpu


def _same(a, b):
    return np.array_equal(a.view(np.int32), b.view(np.int32))


@pytest.fixture(scope="module")
def k64(pg):
    """killeroo at 128x64 (a multiple of the 16-pixel tile), 8 spp: 4 exact-boundary samples."""
    return pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"), xres=128, yres=64, spp=8)


@pytest.fixture(scope="module")
def full(pg, k64):
    with pg.Device(0) as d:
        d.upload(k64)
        st = d.render()
        return d.film(), st


def test_tile_grid_is_film_pixels(pg, k64, full):
    ntx, nty = pg.tile_grid(k64)
    assert (ntx, nty) == (8, 4)          # the sample extent (129 x 65) would give 9 x 5
    with pg.Device(0) as d:
        d.upload(k64)
        with pytest.raises(RuntimeError):
            d.render(tiles=[ntx * nty])
        d.render(tiles=np.arange(ntx * nty))
        assert _same(d.film(), full[0])


def test_repeated_calls_reuse_the_setup(pg, k64, full):
    """A context keeps its last render call's setup (pixel lists, exact-boundary samples and their
    contribution lists) for a call with the same tiles, sample range and scene.
    Alternating tile sets, sample ranges and a scene re-upload must give the films of fresh
    contexts, spills included."""
    ref, st_full = full
    ntx, nty = pg.tile_grid(k64)
    a, b = np.arange(0, ntx * nty, 2), np.arange(1, ntx * nty, 2)
    fresh = {}
    for name, tiles in (("a", a), ("b", b)):
        with pg.Device(0) as d:
            d.upload(k64)
            d.render(tiles=tiles)
            fresh[name] = d.film()
    with pg.Device(0) as d:
        d.upload(k64)
        for name, tiles in (("a", a), ("a", a), ("b", b), ("a", a)):
            st = d.render(tiles=tiles)
            assert _same(d.film(), fresh[name]), name
        for _ in range(2):
            st = d.render()
            assert _same(d.film(), ref)
            assert st[pg.STAT_SPILLS] == st_full[pg.STAT_SPILLS] > 0
        d.render(spp_begin=0, spp_end=3)
        d.render(spp_begin=0, spp_end=8)
        assert _same(d.film(), ref)
        small = pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"), xres=128, yres=64, spp=4)
        d.upload(small)            # a new scene: same tiles and range, other samples
        d.render()
        f4 = d.film()
    with pg.Device(0) as d:
        d.upload(small)
        d.render()
        assert _same(d.film(), f4)


def test_many_spp_batches_and_runs(pg, k64, full, monkeypatch):
    """128x64 px x 32 bands x 4 B = 1 MiB per sample: a 1 MiB budget gives 8 batches of one
    sample; 300 slots give ~27 regenerations per slot per batch."""
    monkeypatch.setenv("PBRTGPU_LBUF_MB", "1")
    monkeypatch.setenv("PBRTGPU_SLOTS", "300")
    with pg.Device(0) as d:
        d.upload(k64)
        st = d.render()
        film = d.film()
    assert st[pg.STAT_PATHS] == full[1][pg.STAT_PATHS]
    assert st[pg.STAT_SPILLS] == full[1][pg.STAT_SPILLS] > 0
    assert st[pg.STAT_PASSES] > 8 * 20
    assert _same(film, full[0])


def test_sample_ranges_accumulate(pg, k64, full):
    ref, st_full = full
    with pg.Device(0) as d:
        d.upload(k64)
        a = d.render(spp_begin=0, spp_end=3)
        b = d.render(spp_begin=3, spp_end=8, accumulate=True)
        film = d.film()
    assert a[pg.STAT_PATHS] + b[pg.STAT_PATHS] == st_full[pg.STAT_PATHS]
    # the exact-boundary samples of each range are still added to their neighbour pixels
    assert a[pg.STAT_SPILLS] + b[pg.STAT_SPILLS] == st_full[pg.STAT_SPILLS] > 0
    den = np.maximum(np.abs(ref).max(axis=2, keepdims=True), 1e-3)
    assert (np.abs(film - ref) / den).max() < 1e-5
    # a pixel's own samples are added in sample order either way
    assert np.all(film.view(np.int32) == ref.view(np.int32), axis=2).mean() > 0.99


def test_render_multi_and_gather(pg, k64, full):
    """Two contexts on one GPU stand in for two GPUs: dealt slices, host gather, and the
    full-frame film bit for bit, for one and for several slices per context."""
    ref = full[0]
    with pg.Device(0) as d0, pg.Device(0) as d1:
        d0.upload(k64)
        d1.upload(k64)
        for slices in (1, 3):
            film, st = pg.render_multi([d0, d1], slices_per_device=slices)
            assert _same(film, ref), slices
            assert st[:, pg.STAT_PATHS].sum() == full[1][pg.STAT_PATHS]
            assert (st[:, pg.STAT_PATHS] > 0).all()
        # a rank's share: slice r of 2, gathered into one shared film
        ntx, nty = pg.tile_grid(k64)
        shared = np.full(ref.shape, -1.0, np.float32)
        for r, d in enumerate((d0, d1)):
            t = pg.tile_slice(ntx * nty, r, 2)
            d.render(tiles=t)
            d.gather(shared, tiles=t)
        assert _same(shared, ref)
        with pytest.raises(RuntimeError):
            pg.render_multi([d0, d0])


def test_serial_mode_same_film(pg, k64, full, monkeypatch):
    monkeypatch.setenv("PBRTGPU_SERIAL", "1")
    with pg.Device(0) as d:
        d.upload(k64)
        d.render()
        assert _same(d.film(), full[0])
        t = d.timing()
        assert t["k_shade"]["ms"] > 0 and t["k_trace_closest"]["ms"] > 0


def test_bench_two_ranks_gather_one_frame(pg, tmp_path):
    """bench.py's multi-process path on real hardware: torch.distributed.run with 2 ranks (on a
    1-GPU box both ranks share the GPU), each rendering its interleaved tile slice and writing
    its pixels into the shared host film -- the gathered film is the single-device film bit
    for bit."""
    import subprocess
    import sys
    from conftest import ROOT
    out = str(tmp_path / "film.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
           "--master-port=%d" % (29500 + os.getpid() % 1000), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "1", "--warmup", "0", "--no-cpu", "--no-roofline", "--res", "96", "--spp", "8", "--dump-film", out]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    import json
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["config"]["shard"] == "tiles" and len(d["per_gpu_ms_per_step"]) == 2
    scene = pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"), xres=96, yres=96, spp=8)
    with pg.Device(0) as dv:
        dv.upload(scene)
        dv.render()
        ref = dv.film()
    assert _same(np.load(out), ref)


def test_instanced_walks_agree_with_work_counters(pg, monkeypatch):
    """k_trace_inst (two-level persistent walk) against the bvh_walk kernels on C5's scene:
    identical per-path radiance, and identical traversal work (rays, nodes visited, primitive
    tests, hits) -- the same nodes and primitives per ray, in the reference's order."""
    scene = pg.Scene.load(os.path.join(PACKS, "anim-killeroos-moving.pack"), xres=64, yres=48, spp=8)
    c = scene.flat.camera
    keys = np.array([(x, y, s) for y in range(c.sy_start, c.sy_end, 3) for x in range(c.sx_start, c.sx_end, 2)
                     for s in range(scene.spp)], np.int32)
    out = {}
    for walk in ("persistent", "legacy"):
        monkeypatch.setenv("PBRTGPU_INST_WALK", walk)
        with pg.Device(0) as d:
            d.upload(scene)
            L = d.trace_paths(keys)
            d.render(count_work=True)
            out[walk] = (L, d.timing()["work"], d.film())
    assert _same(out["persistent"][0], out["legacy"][0])
    assert _same(out["persistent"][2], out["legacy"][2])
    for k in ("rays", "shadow_rays", "nodes_closest", "nodes_shadow", "tris_closest", "tris_shadow", "quads_closest",
              "quads_shadow", "hits"):
        assert out["persistent"][1][k] == out["legacy"][1][k], k
