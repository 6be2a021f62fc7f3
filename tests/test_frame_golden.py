"""Whole-frame parity at the configs' REAL resolution and sample count (BASELINE.json configs 1-5:
C1 in the reference's RGB build; north star: image error vs the CPU reference).

The fixtures (tools/make_frame_golden.py) hold, for every 16x16 tile of the reference harness's
film at full size and spp, a blake2b-64 hash of the tile's float32 bits, its float64 sum and its
largest |value| (a few KB instead of the 63 MB film).  The harness rendered the frame as strips,
each strip's sample window one row larger on each side, so every pixel holds all of its
contributions in the reference's order (spectralImage.cpp:77-152, samplerrenderer.cpp:119-147).

CPU: the glibc-float oracle renders a few tiles (a frame corner, tiles over the light and over
the killeroo) as one-pixel-larger windows: their hashes must be the reference's.
GPU: the whole frame through pbrtgpu_render_tiles; every tile's hash must be the reference's
(bit-exact film), and the mismatching tiles, if any, are reported with their sums.
"""
import json
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PACKS, ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
from make_frame_golden import tile_digest  # noqa: E402

FRAMES = ["killeroo_frame_c2_700x700s256", "anim_frame_c5_600x600s512", "metal_frame_c4_400x400s4096",
          "killeroo_rgb_frame_c1_400x400s64", "bunny_frame_c3_1920x1080s1024"]
# the scene pack of a frame (its name's prefix before "_frame"): C1 is the reference's RGB build
PACK = {"killeroo": "killeroo-simple.pack", "bunny": "bunny.pack", "metal": "metal.pack",
        "anim": "anim-killeroos-moving.pack", "killeroo_rgb": "killeroo-simple-rgb.pack"}
# tiles (tx, ty) the CPU test renders with the oracle: a frame corner, a tile of the right /
# bottom border (partial tiles: 700 = 43 * 16 + 12), and two interior tiles (C3: 1 M paths per
# tile at 1024 spp, so two tiles)
CPU_TILES = {"killeroo": [(0, 0), (43, 43), (5, 2), (7, 19)], "anim": [(0, 0), (37, 37), (8, 16)],
             "metal": [(0, 0), (24, 24), (7, 8)], "killeroo_rgb": [(0, 0), (24, 24), (6, 9), (12, 13)],
             "bunny": [(0, 0), (60, 34)]}


def _key(name):
    return name.split("_frame")[0]
AVAILABLE = [n for n in FRAMES if os.path.exists(os.path.join(GOLDEN, n + ".npz"))]


def _load(pg, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    w, h, spp, seed, md, bands, tile = [int(v) for v in g["config"]]
    scene = pg.Scene.load(os.path.join(PACKS, PACK[_key(name)]), xres=w, yres=h, spp=spp, maxdepth=md,
                          seed=seed)
    assert scene.bands == bands and tile == 16
    return g, scene


def test_frame_fixtures_present():
    assert "killeroo_frame_c2_700x700s256" in AVAILABLE and "anim_frame_c5_600x600s512" in AVAILABLE


@pytest.mark.parametrize("name", AVAILABLE)
def test_frame_fixture_shape(name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    W, H = [int(v) for v in g["config"][:2]]
    assert g["hash"].shape == ((H + 15) // 16, (W + 15) // 16) == g["sum"].shape == g["absmax"].shape
    assert np.isfinite(g["sum"]).all() and g["sum"].sum() > 0
    assert len(np.unique(g["hash"])) > g["hash"].size // 2   # tiles differ: not a hash of empty films


@pytest.mark.parametrize("name", AVAILABLE)
def test_frame_tiles_oracle_bit_exact_vs_reference(pg, name):
    """The glibc-float oracle renders a few tiles of the full-size frame at full spp (every sample
    of a window one pixel larger): their hashes are the reference frame's."""
    g, scene = _load(pg, name)
    o = pg.oracle(libm_float=True)
    for tx, ty in CPU_TILES[_key(name)]:
        x0, y0 = 16 * tx, 16 * ty
        x1, y1 = min(x0 + 16, scene.width), min(y0 + 16, scene.height)
        film, _ = o.render(scene, window=(x0 - 1, x1 + 1, y0 - 1, y1 + 1), threads=min(16, os.cpu_count() or 8))
        crop = np.zeros((16, 16, scene.bands), np.float32)[:y1 - y0, :x1 - x0]
        crop[:] = film[y0:y1, x0:x1]
        hs, sm, _ = tile_digest(crop)
        assert hs[0, 0] == g["hash"][ty, tx], (name, tx, ty, sm[0, 0], g["sum"][ty, tx])


@pytest.mark.gpu
@pytest.mark.parametrize("name", AVAILABLE)
def test_frame_gpu_bit_exact_vs_reference(pg, name):
    """The whole frame on the GPU: every 16x16 tile's float32 bits hash to the reference's."""
    g, scene = _load(pg, name)
    with pg.Device(0) as d:
        d.upload(scene)
        st = d.render()
        film = d.film()
    assert st[pg.STAT_PATHS] == scene.width * scene.height * scene.spp
    hs, sm, mx = tile_digest(film)
    bad = np.argwhere(hs != g["hash"])
    rel = np.abs(sm - g["sum"]) / np.maximum(np.abs(g["sum"]), 1e-30)
    rec = {"name": name, "tiles": int(hs.size), "tiles_differing": int(len(bad)),
           "max_tile_sum_rel": float(rel.max()), "first_bad": [[int(a), int(b)] for a, b in bad[:8]],
           "spills": float(st[pg.STAT_SPILLS])}
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "frame_parity.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    print(rec)
    assert len(bad) == 0, rec
