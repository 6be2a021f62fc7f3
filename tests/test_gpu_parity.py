"""GPU parity: the HIP path (libpbrtgpu.so, through the C ABI) against the CPU oracle and the
reference harness's own fixtures.

The oracle here is oracle/liboracle.so, whose float transcendentals are glibc 2.35's routines
restated (include/pbrt_libmf.h, checked over all 2^32 inputs against the system libm), the same
header the kernels compile; it is pinned bit-exactly to the reference harness by
tests/test_oracle_golden.py.  Every assertion here is bit equality of the float32 results (NaN as
NaN, conftest.assert_bit_exact): per-path radiance, films, hit records, occlusion answers.  The
lens camera's results are pinned to the oracle only (its reference TU needs GSL, absent here:
parity unpinned vs the reference).
"""
import os

import numpy as np

from conftest import assert_bit_exact
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pg, killeroo64):
    d = pg.Device(0)
    d.upload(killeroo64)
    yield d
    d.close()


def _keys(scene, stride=1):
    c = scene.flat.camera
    ks = [(x, y, s) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
          for s in range(scene.spp)]
    return np.array(ks[::stride], dtype=np.int32)


def test_native_library_loaded(pg):
    lib = pg.gpu_lib()
    assert lib.pbrtgpu_device_count() >= 1
    assert lib.pbrtgpu_abi_version() == pg.ABI_VERSION


def test_paths_match_oracle(pg, killeroo64, dev):
    keys = _keys(killeroo64)
    Lg = dev.trace_paths(keys)
    Lo = pg.oracle().trace_paths(killeroo64, keys)
    assert_bit_exact(Lg, Lo, "paths vs oracle")


def test_film_matches_oracle(pg, killeroo64, dev):
    st = dev.render()
    film = dev.film()
    ref, ost = pg.oracle().render(killeroo64)
    assert st[pg.STAT_PATHS] == killeroo64.width * killeroo64.height * killeroo64.spp
    assert_bit_exact(film, ref, "film vs oracle")


def test_intersect_matches_oracle(pg, killeroo64, dev):
    rng = np.random.RandomState(12345)
    n = 20000
    lo = np.array([-1000, -1000, -140], np.float32)
    hi = np.array([1000, 1000, 200], np.float32)
    o = lo + (hi - lo) * rng.rand(n, 3).astype(np.float32)
    d = rng.randn(n, 3).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d, np.zeros((n, 1), np.float32), np.full((n, 1), np.inf, np.float32)], axis=1)
    hg, og = dev.intersect(rays)
    ho, oo = pg.oracle().intersect(killeroo64, rays)
    assert np.array_equal(hg[:, 3].view(np.int32), ho[:, 3].view(np.int32))
    assert np.array_equal(hg[:, 0].view(np.int32), ho[:, 0].view(np.int32))
    assert np.array_equal(og, oo)


def test_regeneration_small_slot_pool(pg, killeroo64, dev, monkeypatch):
    """Few path slots -> many regenerations per slot; results must not depend on it."""
    keys = _keys(killeroo64, stride=3)
    ref = dev.trace_paths(keys)
    monkeypatch.setenv("PBRTGPU_SLOTS", "257")
    small = dev.trace_paths(keys)
    assert np.array_equal(ref.view(np.int32), small.view(np.int32))
    st = dev.render()
    film = dev.film()
    monkeypatch.delenv("PBRTGPU_SLOTS")
    dev.render()
    assert np.array_equal(film.view(np.int32), dev.film().view(np.int32))
    assert st[pg.STAT_PASSES] > 20


def test_work_counters(pg, killeroo64, dev):
    dev.render(count_work=True)
    w = dev.timing()["work"]
    n = killeroo64.width * killeroo64.height * killeroo64.spp
    assert w["rays"] >= n                      # at least one camera ray per path
    assert w["nodes_closest"] > w["rays"]
    assert 0 < w["hits"] <= w["rays"]


def _golden_scene(pg, cfg, name="killeroo"):
    from conftest import PACKS
    w, h, spp, seed, md = [int(v) for v in cfg]
    pack = {"anim": "anim-killeroos-moving.pack", "bunny": "bunny.pack", "metal": "metal.pack",
            "coverage": "coverage.pack", "imagemap": "imagemap.pack",
            "animcam": "animcam.pack", "textured": "textured.pack", "envmap": "envmap.pack", "lights": "lights.pack",
            "ortho": "ortho.pack", "heightfield": "heightfield.pack",
            "cylinder": "cylinder.pack", "anisoward": "anisoward.pack", "mappings": "mappings.pack", "checker": "checker.pack",
            "shinymetal": "shinymetal.pack", "nurbs": "nurbs.pack"}.get(name.split("_")[0],
                                                                                              "killeroo-simple.pack")
    if "_b30_" in name:
        pack = pack.replace(".pack", "-b30.pack")
    return pg.Scene.load(os.path.join(PACKS, pack), xres=w, yres=h, spp=spp, maxdepth=md, seed=seed)


@pytest.mark.parametrize("name", ["killeroo_paths_64x64s4", "killeroo_paths_48x48s8_seed7_md7", "anim_paths_48x48s4",
                                  "bunny_paths_64x36s4", "metal_paths_48x48s4",
                                  "coverage_paths_64x48s8", "killeroo_keys_c2_700x700s256",
                                  "bunny_keys_c3_1920x1080s1024", "metal_keys_c4_400x400s4096",
                                  "anim_keys_c5_600x600s512", "killeroo_b30_paths_48x40s4",
                                  "coverage_b30_paths_48x36s4", "imagemap_paths_64x48s4",
                                  "imagemap_paths_96x72s2_seed5", "animcam_paths_64x48s4", "textured_paths_64x48s4", "envmap_paths_64x48s4",
                                  "lights_paths_64x48s4", "ortho_paths_64x48s4", "heightfield_paths_64x48s4",
         "cylinder_paths_64x48s4", "anisoward_paths_64x48s4", "mappings_paths_64x48s4", "checker_paths_64x48s4",
         "shinymetal_paths_64x48s4", "nurbs_paths_64x48s4"])
def test_paths_vs_reference_golden(pg, name):
    """GPU against the reference harness's own per-path radiance (fixed seeds); the *_keys_*
    fixtures are the configs at their real resolution and sample count."""
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = _golden_scene(pg, g["config"], name)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
    assert_bit_exact(L, g["L"], name)


@pytest.mark.parametrize("name", ["killeroo_film_96x72s16", "anim_film_40x40s8", "bunny_film_48x27s8",
                                  "metal_film_40x40s8", "coverage_film_64x48s8", "killeroo_b30_film_40x32s8",
                                  "coverage_b30_film_40x30s4", "imagemap_film_64x48s8",
                                  "animcam_film_64x48s4", "textured_film_64x48s8", "envmap_film_64x48s8",
                                  "lights_film_64x48s8", "ortho_film_64x48s4", "heightfield_film_64x48s4",
                                  "cylinder_film_64x48s4", "anisoward_film_64x48s4", "mappings_film_64x48s4", "checker_film_64x48s4",
                                  "shinymetal_film_64x48s4", "nurbs_film_64x48s4"])
def test_film_vs_reference_golden(pg, name):
    """Whole-film render against the reference's film (raw sums, incl. neighbour-pixel
    samples): bit for bit."""
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = _golden_scene(pg, g["config"], name)
    with pg.Device(0) as d:
        d.upload(scene)
        st = d.render()
        film = d.film()
    ref = g["film"]
    if name.startswith("killeroo_film"):
        assert st[pg.STAT_SPILLS] > 0
    assert_bit_exact(film, ref, name)


def test_tile_shards_compose_to_full_frame(pg, killeroo64, dev):
    """Rendering tile subsets (as ranks do under --shard tiles) and accumulating them gives
    the full-frame film bit for bit."""
    dev.render()
    full = dev.film()
    ntx, nty = pg.tile_grid(killeroo64)
    ntiles = ntx * nty
    dev.render(tiles=np.arange(0, ntiles, 2))
    dev.render(tiles=np.arange(1, ntiles, 2), accumulate=True)
    assert np.array_equal(full.view(np.int32), dev.film().view(np.int32))


def test_sample_range_split_and_bad_arguments(pg, killeroo64, dev):
    with pytest.raises(RuntimeError):
        dev.render(spp_begin=3, spp_end=2)
    with pytest.raises(RuntimeError):
        dev.render(tiles=[10 ** 6])
    with pytest.raises(RuntimeError):
        dev.trace_paths(np.array([[10 ** 5, 0, 0]], np.int32))


@pytest.mark.parametrize("walk", ["persistent", "legacy"])
def test_motion_blur_instances_match_oracle(pg, monkeypatch, walk):
    """C5: animated TransformedPrimitives over nested BVHs -- GPU against the oracle, path
    by path and film, bit for bit (same transcendental definition); the two-level persistent
    traversal kernel (k_trace_inst, default) and the one-ray-per-thread bvh_walk kernels
    (PBRTGPU_INST_WALK=legacy)."""
    from conftest import PACKS
    monkeypatch.setenv("PBRTGPU_INST_WALK", walk)
    scene = pg.Scene.load(os.path.join(PACKS, "anim-killeroos-moving.pack"), xres=40, yres=40, spp=4)
    assert scene.flat.n_instances == 2
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        Lg = d.trace_paths(keys)
        d.render()
        film = d.film()
        rays = np.zeros((2000, 8), np.float32)
        rng = np.random.RandomState(7)
        rays[:, :3] = rng.uniform(-300, 300, (2000, 3))
        dd = rng.randn(2000, 3)
        rays[:, 3:6] = dd / np.linalg.norm(dd, axis=1, keepdims=True)
        rays[:, 7] = np.inf
        hg, og = d.intersect(rays)
    o = pg.oracle()
    Lo = o.trace_paths(scene, keys)
    assert_bit_exact(Lg, Lo, "paths vs oracle")
    ref, _ = o.render(scene)
    assert_bit_exact(film, ref, "film vs oracle")
    ho, oo = o.intersect(scene, rays)
    assert np.array_equal(hg[:, 3].view(np.int32), ho[:, 3].view(np.int32))
    assert np.array_equal(og, oo)


@pytest.mark.parametrize("kd_lds", ["1", "0"])
def test_measured_brdf_matches_oracle(pg, monkeypatch, kd_lds):
    """C3: measured (mystique) BRDF through the kd-tree, point light, disk light -- GPU
    against the oracle path by path and film; kd-tree walk over the LDS copy of the tree
    (default) and over global memory (PBRTGPU_KD_LDS=0, trees too large for LDS)."""
    from conftest import PACKS
    monkeypatch.setenv("PBRTGPU_KD_LDS", kd_lds)
    scene = pg.Scene.load(os.path.join(PACKS, "bunny.pack"), xres=48, yres=27, spp=4)
    assert scene.flat.n_kdnodes > 0
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        Lg = d.trace_paths(keys)
        d.render()
        film = d.film()
    o = pg.oracle()
    Lo = o.trace_paths(scene, keys)
    assert_bit_exact(Lg, Lo, "paths vs oracle")
    ref, _ = o.render(scene)
    assert_bit_exact(film, ref, "film vs oracle")


def test_metal_textures_environment_match_oracle(pg):
    """C4 (60 bands): FresnelConductor metal, imagemap-textured substrate with a textured bump
    (EWA lookups with camera ray differentials), infinite light -- GPU against the oracle."""
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, "metal.pack"), xres=40, yres=40, spp=4)
    assert scene.bands == 60
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        Lg = d.trace_paths(keys)
        d.render()
        film = d.film()
    o = pg.oracle()
    Lo = o.trace_paths(scene, keys)
    assert_bit_exact(Lg, Lo, "paths vs oracle")
    ref, _ = o.render(scene)
    assert_bit_exact(film, ref, "film vs oracle")


def test_shade_variants_agree(pg, killeroo64, monkeypatch):
    """The feature-specialised shade kernel (no measured BRDF / textures / environment light)
    and the full kernel give the same film bit for bit on a scene both can render."""
    with pg.Device(0) as d:
        d.upload(killeroo64)
        d.render()
        lean = d.film()
    monkeypatch.setenv("PBRTGPU_SHADE_FULL", "1")
    with pg.Device(0) as d:
        d.upload(killeroo64)
        d.render()
        full = d.film()
    assert np.array_equal(lean.view(np.int32), full.view(np.int32))


@pytest.mark.parametrize("pack,integ", [("killeroo-simple-b60.pack", "directlighting"), ("killeroo-simple.pack", "directlighting"),
                                        ("killeroo-simple-rgb.pack", "path"), ("killeroo-simple.pack", "path")])
def test_basic_material_objects_match_oracle(pg, monkeypatch, pack, integ):
    """Scenes whose materials are all matte / plastic run the FEAT_BASIC shading objects (the other
    BxDF kinds compiled out: path integrator at 32 and 3 bands, DirectLighting at 32 and 60): per
    path and film bit-exact against the oracle, and the film equal to the lean (FEAT 0) objects'."""
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, pack), xres=40, yres=32, spp=2, maxdepth=5, integrator=integ)
    keys = _keys(scene, stride=3)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(keys)
        d.render()
        film = d.film()
        assert d.timing()["shade_feat"] == 8   # FEAT_BASIC
    o = pg.oracle()
    assert np.any(L != 0)
    assert_bit_exact(L, o.trace_paths(scene, keys), "paths vs oracle")
    ref, _ = o.render(scene)
    assert_bit_exact(film, ref, "film vs oracle")
    monkeypatch.setenv("PBRTGPU_SHADE_FULL", "1")   # the all-features objects
    with pg.Device(0) as d:
        d.upload(scene)
        d.render()
        full = d.film()
    assert np.array_equal(film.view(np.int32), full.view(np.int32))


def test_coverage_scene_matches_oracle(pg):
    """tests/scenes/coverage.pbrt: glass, mirror, Oren-Nayar, copper with textured bump,
    textures, three light types -- GPU against the oracle path by path and film."""
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"))
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        Lg = d.trace_paths(keys)
        d.render()
        film = d.film()
    o = pg.oracle()
    Lo = o.trace_paths(scene, keys)
    assert_bit_exact(Lg, Lo, "paths vs oracle")
    ref, _ = o.render(scene)
    assert_bit_exact(film, ref, "film vs oracle")


@pytest.mark.parametrize("ring,refill", [("1", "1"), ("2", "64"), ("4", "7")])
def test_traversal_stack_spill_and_ray_replacement(pg, killeroo64, dev, monkeypatch, ring, refill):
    """k_trace_pt keeps the top of each lane's traversal stack in an LDS ring and spills the
    rest to HBM, and replaces finished rays once `refill` lanes idle.  Tiny rings (every
    deep push spills) and extreme thresholds must give the default's radiance bit for bit."""
    keys = _keys(killeroo64, stride=2)
    ref = dev.trace_paths(keys)
    monkeypatch.setenv("PBRTGPU_STACK_LDS", ring)
    monkeypatch.setenv("PBRTGPU_REFILL", refill)
    with pg.Device(0) as d:
        d.upload(killeroo64)
        got = d.trace_paths(keys)
        d.render(count_work=True)
        w = d.timing()["work"]
    dev.render(count_work=True)
    w0 = dev.timing()["work"]
    assert np.array_equal(ref.view(np.int32), got.view(np.int32))
    for k in ("rays", "shadow_rays", "nodes_closest", "nodes_shadow", "tris_closest", "tris_shadow", "hits"):
        assert w[k] == w0[k], k


@pytest.mark.parametrize("name", ["bunny", "coverage"])
def test_mis_rays_that_can_reach_the_light_are_traced(pg, name):
    """k_shade skips only MIS rays that miss every shape of the sampled area light
    (wavefront.h mis_may_reach).  In scenes whose BSDF samples do reach the light some MIS
    rays are still traced, and per-path radiance stays identical to the oracle, which traces
    every MIS ray."""
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, name + ".pack"), xres=48, yres=32, spp=8)
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        d.render(count_work=True)
        w = d.timing()["work"]
        Lg = d.trace_paths(keys)
    assert w["mis_rays"] > 0
    Lo = pg.oracle().trace_paths(scene, keys)
    assert_bit_exact(Lg, Lo, name)


def test_regular_halfangle_brdf_vs_reference_golden(pg, merl_dir):
    """GPU RegularHalfangleBRDF against the reference harness's per-path radiance and film
    (tests/scenes/merl.pbrt with the synthetic MERL table), bit for bit."""
    from conftest import GOLDEN, merl_scene
    g = np.load(os.path.join(GOLDEN, "merl_paths_64x48s8.npz"))
    scene = merl_scene(pg, merl_dir, g["config"])
    gf = np.load(os.path.join(GOLDEN, "merl_film_64x48s8.npz"))
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
        d.render()
        film = d.film()
    assert_bit_exact(L, g["L"], "merl paths vs reference")
    assert_bit_exact(film, gf["film"], "merl film vs reference")
    assert_bit_exact(L, pg.oracle().trace_paths(scene, g["keys"]), "merl paths vs oracle")


DL = ["checker_dl_%s_48x36s4", "mappings_dl_%s_48x36s4", "shinymetal_dl_%s_48x36s4", "anisoward_dl_%s_48x36s4", "cylinder_dl_%s_48x36s4", "ortho_dl_%s_48x36s4", "lights_dl_%s_48x36s4", "textured_dl_%s_48x36s4", "envmap_dl_%s_48x36s4", "killeroo_dl_%s_48x40s4", "bunny_dl_%s_48x27s4", "anim_dl_%s_40x40s4", "coverage_dl_%s_64x48s4",
      "coverage_dlone_%s_64x48s4"]


@pytest.mark.parametrize("base", DL)
def test_direct_lighting_vs_reference_golden(pg, base):
    """DirectLightingIntegrator on the GPU (directlighting.h: light samples one pass each,
    SpecularReflect / SpecularTransmit as a per-slot frame stack) against the reference
    harness's per-path radiance and film, and path by path against the oracle."""
    from conftest import GOLDEN
    from test_oracle_golden import dl_scene
    g = np.load(os.path.join(GOLDEN, base % "paths" + ".npz"))
    gf = np.load(os.path.join(GOLDEN, base % "film" + ".npz"))
    scene = dl_scene(pg, g, base % "paths")
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
        d.render()
        film = d.film()
    assert_bit_exact(L, g["L"], base % "paths")
    assert_bit_exact(film, gf["film"], base % "film")
    assert_bit_exact(L, pg.oracle().trace_paths(scene, g["keys"]), base + " vs oracle")


@pytest.mark.parametrize("strategy,md", [("all", 6), ("one", 3)])
def test_direct_lighting_recursion_and_regeneration(pg, monkeypatch, strategy, md):
    """Deep specular recursion (coverage.pbrt's glass and mirror, maxdepth up to 6: every
    vertex may push both children) and a tiny slot pool (many regenerations per slot) give the
    oracle's radiance; the film does not depend on the slot count."""
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=md,
                          integrator="directlighting", strategy=strategy)
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(keys)
        d.render()
        film = d.film()
        assert np.array_equal(L.view(np.int32), d.trace_paths(keys).view(np.int32))   # deterministic
        monkeypatch.setenv("PBRTGPU_SLOTS", "193")
        Ls = d.trace_paths(keys)
        d.render()
        films = d.film()
    assert np.array_equal(L.view(np.int32), Ls.view(np.int32))
    assert np.array_equal(film.view(np.int32), films.view(np.int32))
    assert_bit_exact(L, pg.oracle().trace_paths(scene, keys), "paths vs oracle")


def test_rng_sequence_matches_reference(pg):
    """The device RNG (5-word window for outputs 0-226, then the full state rebuilt and twisted
    every 624 outputs) against the oracle's MT19937, itself pinned to the reference's
    (test_oracle_golden.py), over 4 generations."""
    ora = pg.oracle()
    with pg.Device(0) as d:
        for seed in (0, 1, 5489, 123456789, 0xdeadbeef):
            assert np.array_equal(d.mt_sequence(seed, 2600), ora.mt_first(seed, 2600))


@pytest.mark.parametrize("integ,md,strategy", [("directlighting", 16, "all"), ("directlighting", 20, "one"),
                                               ("path", 60, None)])
def test_deep_paths_past_the_first_rng_block(pg, integ, md, strategy):
    """maxdepth beyond the first MT19937 block: DirectLighting's specular recursion on
    coverage.pbrt's glass and mirrors at maxdepth 16 / 20 draws up to ~300 values per path, so
    paths continue on the rebuilt full state; the path integrator at maxdepth 60.  Oracle bits."""
    from conftest import PACKS
    kw = dict(integrator=integ, strategy=strategy) if strategy else {}
    scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=md, **kw)
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(keys)
    assert_bit_exact(L, pg.oracle().trace_paths(scene, keys), "paths vs oracle")


@pytest.mark.parametrize("integ,strategy,md", [("directlighting", "all", 6), ("directlighting", "one", 4),
                                               ("path", None, 5)])
def test_independent_of_unwritten_state_and_slot_layout(pg, monkeypatch, integ, strategy, md):
    """PBRTGPU_POISON fills every path-slot array (and the traversal stack spill area) with a byte
    before each run, so a read of state no pass wrote changes the radiance; the slot pool size
    changes which items share a wave and in what order slots are regenerated.  Every combination
    gives the same bits, and the oracle's (the DirectLighting non-determinism of
    the first 3-wave build)."""
    from conftest import PACKS
    kw = dict(integrator=integ, strategy=strategy) if strategy else {}
    scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=md, **kw)
    keys = _keys(scene)
    runs = []
    with pg.Device(0) as d:
        d.upload(scene)
        for poison in ("0x00", "0xff", "0x7f"):
            for slots in (None, "193", "4096"):
                monkeypatch.setenv("PBRTGPU_POISON", poison)
                if slots: monkeypatch.setenv("PBRTGPU_SLOTS", slots)
                else: monkeypatch.delenv("PBRTGPU_SLOTS", raising=False)
                runs.append(d.trace_paths(keys))
    for r in runs[1:]:
        assert np.array_equal(r.view(np.int32), runs[0].view(np.int32))
    assert_bit_exact(runs[0], pg.oracle().trace_paths(scene, keys), "paths vs oracle")


@pytest.mark.parametrize("integ,strategy,md", [("directlighting", "all", 6), ("path", None, 5), ("path", None, 24)])
def test_drain_list_mode_is_exact(pg, monkeypatch, integ, strategy, md):
    """The drain on a live-slot list (once the items are all taken, k_shade and the
    DirectLighting kernels take the live slots of k_live_list; the per-wave compaction becomes the
    identity) against the same runs with it off (PBRTGPU_DRAIN_LIST=0): films and per-path
    radiance bit for bit, with slot pools small enough that most passes run in list mode (193
    slots: many drains of a few waves) and one large pool; and the drain's tail kernel (k_tail:
    the last paths run to their end in one launch) off and switched on as early as allowed."""
    from conftest import PACKS
    kw = dict(integrator=integ, strategy=strategy) if strategy else {}
    scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=md, **kw)
    keys = _keys(scene)
    out = {}
    with pg.Device(0) as d:
        d.upload(scene)
        for slots in ("193", "4096"):
            monkeypatch.setenv("PBRTGPU_SLOTS", slots)
            for on in ("1", "0"):
                monkeypatch.setenv("PBRTGPU_DRAIN_LIST", on)
                d.render()
                out[(slots, on)] = (d.film(), d.trace_paths(keys))
        # the drain's tail kernel (k_tail, path integrator): off, and on from the first eligible pass
        for tail in ("0", "100000000"):
            monkeypatch.setenv("PBRTGPU_DRAIN_LIST", "1")
            monkeypatch.setenv("PBRTGPU_SLOTS", "4096")
            monkeypatch.setenv("PBRTGPU_TAIL", tail)
            d.render()
            out[("tail", tail)] = (d.film(), d.trace_paths(keys))
        monkeypatch.delenv("PBRTGPU_TAIL")
    ref = out[("4096", "0")]
    for k, (film, paths) in out.items():
        assert np.array_equal(film.view(np.int32), ref[0].view(np.int32)), k
        assert np.array_equal(paths.view(np.int32), ref[1].view(np.int32)), k
    assert_bit_exact(ref[1], pg.oracle().trace_paths(scene, keys), "paths vs oracle")


@pytest.mark.parametrize("name", ["killeroo_keys_c2_700x700s256", "killeroo_film_96x72s16", "killeroo_dl_paths_48x40s4",
                                  "killeroo_dl_film_48x40s4", "coverage_paths_64x48s8"])
def test_quantized_shadow_walk_vs_reference_golden(pg, monkeypatch, name):
    """The opt-in quantized 4-wide shadow walk (PBRTGPU_SHADOW4Q=1, k_trace_s4q: 64-byte nodes with
    conservative outer / inner boxes, a leaf's hit kept only when its exact ancestors pass) against
    the reference harness: per path and film, bit for bit, path integrator and DirectLighting."""
    from conftest import GOLDEN
    from test_oracle_golden import dl_scene
    monkeypatch.setenv("PBRTGPU_SHADOW4Q", "1")
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = dl_scene(pg, g, name) if "_dl_" in name else _golden_scene(pg, g["config"], name)
    with pg.Device(0) as d:
        d.upload(scene)
        if "film" in name:
            d.render()
            assert_bit_exact(d.film(), g["film"], name)
        else:
            assert_bit_exact(d.trace_paths(g["keys"]), g["L"], name)


META = ["metadata_material_%s_48x36s4", "metadata_mesh_%s_48x36s4", "metadata_depth_%s_48x36s4",
        "killeroo_meta_mesh_%s_40x32s2", "anim_meta_mesh_%s_40x32s2", "bunny_meta_depth_%s_40x32s2",
        "heightfield_meta_mesh_%s_48x36s2", "nurbs_meta_mesh_%s_48x36s2"]


@pytest.mark.parametrize("base", META)
def test_metadata_vs_reference_golden(pg, base):
    """MetadataIntegrator on the GPU (metadata.h: one pass per camera sample) against the
    reference harness and the oracle, bit for bit: hits (ids, depth = one sqrt of the hit
    distance) and camera rays that miss into metadata.pbrt's environment light (its Le)."""
    from conftest import GOLDEN
    from test_oracle_golden import meta_scene
    g = np.load(os.path.join(GOLDEN, base % "paths" + ".npz"))
    gf = np.load(os.path.join(GOLDEN, base % "film" + ".npz"))
    scene = meta_scene(pg, g, base % "paths")
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
        d.render()
        film = d.film()
    assert_bit_exact(L, g["L"], base % "paths")
    assert_bit_exact(film, gf["film"], base % "film")
    o = pg.oracle()
    assert_bit_exact(L, o.trace_paths(scene, g["keys"]), "paths vs oracle")
    of, _ = o.render(scene)
    assert_bit_exact(film, of, "film vs oracle")


SPEC = ["killeroo_spec32_%s_40x32s4", "coverage_spec3_%s_48x36s4", "coverage_specsampler8_%s_48x36s8",
        "killeroo_spec5_dl_%s_32x24s2", "killeroo_b30_spec5_%s_32x24s4", "coverage_b30_specsampler6_%s_40x30s8"]


@pytest.mark.parametrize("base", SPEC)
def test_spectral_renderer_vs_reference_golden(pg, base):
    """SpectralRenderer on the GPU (singleDirection: nWaveBands paths per camera sample, each
    writing its band's indices of the sample's row, then k_spec_guard; samplerDirection: band
    s % nWaveBands) against the reference harness's per-sample spectra and film, and sample by
    sample against the oracle."""
    from conftest import GOLDEN
    from test_oracle_golden import spec_scene
    g = np.load(os.path.join(GOLDEN, base % "paths" + ".npz"))
    gf = np.load(os.path.join(GOLDEN, base % "film" + ".npz"))
    scene = spec_scene(pg, g, base % "paths")
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
        d.render()
        film = d.film()
    assert_bit_exact(L, g["L"], base % "paths")
    assert_bit_exact(film, gf["film"], base % "film")
    assert_bit_exact(L, pg.oracle().trace_paths(scene, g["keys"]), base + " vs oracle")


def test_spectral_renderer_lanes_batches_and_rejects(pg, monkeypatch):
    """The bands of a sample land in its row whatever lane, slot or Lbuf batch traces them: a
    tiny slot pool and a tiny Lbuf give the same samples and film bit for bit; nWaveBands whose
    band reads past the spectrum (60 bands at the default 32 wave bands, spectrum.h:397) and
    unknown sampling methods are refused."""
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=6,
                          renderer="spectral", wave_bands=7, sampling="single")
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(keys)
        d.render()
        film = d.film()
        monkeypatch.setenv("PBRTGPU_SLOTS", "193")
        monkeypatch.setenv("PBRTGPU_LBUF_MB", "1")
        Ls = d.trace_paths(keys)
        d.render()
        films = d.film()
        assert np.array_equal(L.view(np.int32), Ls.view(np.int32))
        assert np.array_equal(film.view(np.int32), films.view(np.int32))
        assert_bit_exact(L, pg.oracle().trace_paths(scene, keys), "paths vs oracle")
        m = pg.Scene.load(os.path.join(PACKS, "metal.pack"), xres=8, yres=8, spp=1, renderer="spectral")
        assert m.flat.n_bands == 60 and m.flat.wave_bands == 32
        with pytest.raises(RuntimeError, match="past the spectrum"):
            d.upload(m)
        scene.flat.spectral_sampling = 5
        with pytest.raises(RuntimeError, match="sampling"):
            d.upload(scene)


@pytest.mark.parametrize("scene_file,kw", [
    ("lens.pbrt", dict()), ("lens.pbrt", dict(integrator="directlighting")),
    ("lens.pbrt", dict(renderer="spectral", wave_bands=8, sampling="single")),
    ("lens.pbrt", dict(renderer="spectral", wave_bands=10, sampling="sampler")),
    ("lens_diffraction.pbrt", dict()),
    ("lens_diffraction.pbrt", dict(renderer="spectral", wave_bands=8, sampling="single")),
    ("lens_diffraction.pbrt", dict(renderer="spectral", wave_bands=10, sampling="sampler", integrator="directlighting")),
    ("lens_animated.pbrt", dict()),
    ("lens_animated.pbrt", dict(renderer="spectral", wave_bands=8, sampling="single", integrator="directlighting"))])
def test_realistic_diffraction_camera_vs_oracle(pg, monkeypatch, scene_file, kw):
    """RealisticDiffractionCamera (tests/scenes/lens.pbrt: a double-Gauss lens, chromatic
    aberration on, so every SpectralRenderer band refracts with its own n) on the GPU against
    the oracle, sample by sample and film.  PARITY UNPINNED vs the reference: the camera's TU
    includes GSL headers this image lacks.  About 60 % of the camera rays are
    blocked by the stop (weight 0: radiance 0 without a trace); the differentials come from the
    rays one pixel over (camera.cpp:52-81), which the textured materials use.  A tiny slot pool
    gives the same bits.  lens_diffraction.pbrt: diffraction on (realisticDiffraction.cpp:
    1057-1150), the Gaussian drawn from each camera sample's own stream, also
    re-derived for the first hit's differentials."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    scene = pg.Scene.load(os.path.join(here, scene_file), xres=40, yres=30, spp=4, maxdepth=5, **kw)
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(keys)
        d.render()
        film = d.film()
        monkeypatch.setenv("PBRTGPU_SLOTS", "193")
        Ls = d.trace_paths(keys)
    assert np.array_equal(L.view(np.int32), Ls.view(np.int32))
    o = pg.oracle()
    Lo = o.trace_paths(scene, keys)
    zero = ~np.any(Lo != 0, axis=1)
    assert 0.3 < zero.mean() < 0.8                       # blocked camera rays (and the GPU agrees)
    assert np.array_equal(zero, ~np.any(L != 0, axis=1))
    assert_bit_exact(L, Lo, "paths vs oracle")
    of, _ = o.render(scene)
    assert_bit_exact(film, of, "film vs oracle")


@pytest.mark.parametrize("scene_file,kw", [
    ("lens_pinholes.pbrt", dict()),
    ("lens_pinholes.pbrt", dict(renderer="spectral", wave_bands=8, sampling="single")),
    ("lens_microlens.pbrt", dict()),
    ("lens_microlens.pbrt", dict(renderer="spectral", wave_bands=4, sampling="single", integrator="directlighting")),
    ("eye.pbrt", dict()),
    ("eye.pbrt", dict(renderer="spectral", wave_bands=8, sampling="single")),
    ("eye.pbrt", dict(renderer="spectral", wave_bands=10, sampling="sampler", integrator="directlighting"))])
def test_light_field_and_eye_cameras_vs_oracle(pg, scene_file, kw):
    """The RealisticDiffractionCamera's light-field modes and the Gullstrand eye on the GPU
    against the oracle, sample by sample and film, at the scenes' own film size (the pinhole
    array depends on it): an 8 x 6 pinhole array (realisticDiffraction.cpp:248-304, 560-629),
    the same with a two-surface microlens per pinhole and diffraction on every surface
    (:614-876), and IORforEyeEnabled (:196-205, 357-377: under the SpectralRenderer each band
    refracts with the ocular media's IOR at its wavelength).  PARITY UNPINNED vs the reference
    (the camera's TU needs GSL); the device source is also replayed on the CPU
    against the oracle (tests/test_hostsan.py)."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    scene = pg.Scene.load(os.path.join(here, scene_file), spp=4, maxdepth=5, **kw)
    keys = _keys(scene)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(keys)
        d.render()
        film = d.film()
    o = pg.oracle()
    Lo = o.trace_paths(scene, keys)
    assert np.any(Lo != 0)
    assert_bit_exact(L, Lo, "paths vs oracle")
    of, _ = o.render(scene)
    assert_bit_exact(film, of, "film vs oracle")


@pytest.mark.parametrize("name", ["killeroo_rgb_paths_48x40s4", "killeroo_rgb_keys_c1_400x400s64"])
def test_rgb_build_vs_reference_golden(pg, name):
    """C1 (BASELINE configs[0]): the RGBSpectrum build (3 channels, NB = 3 kernels) against the
    reference's RGB harness per path -- keys at C1's 400x400 at 64 spp included -- and the film,
    and against the oracle."""
    from conftest import GOLDEN
    from test_oracle_golden import rgb_scene
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = rgb_scene(pg, g)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
        film = None
        if "paths" in name:
            gf = np.load(os.path.join(GOLDEN, "killeroo_rgb_film_40x32s8.npz"))
            fs = rgb_scene(pg, gf)
            d.upload(fs)
            d.render()
            film = d.film()
    assert_bit_exact(L, g["L"], name)
    assert_bit_exact(L, pg.oracle().trace_paths(scene, g["keys"]), name + " vs oracle")
    if film is not None:
        assert_bit_exact(film, gf["film"], "killeroo_rgb_film_40x32s8")


@pytest.mark.parametrize("name", ["imagemap_rgb_paths_64x48s4", "textured_rgb_paths_64x48s4", "envmap_rgb_paths_64x48s4",
                                  "coverage_rgb_paths_64x48s4", "merl_rgb_paths_64x48s4", "lights_rgb_paths_64x48s4",
                                  "envmap_rgb_dl_paths_48x36s4",
                                  "coverage_rgb_dl_paths_48x36s4"])
def test_rgb_build_features_vs_reference_golden(pg, name, request):
    """The RGB build's image textures, normal maps, textured parameters, environment map, SPD
    spectra and MERL tables (NB = 3 kernels, FromRGB the identity) against the brgb harness per
    path and film, bit for bit."""
    from conftest import GOLDEN
    from test_oracle_golden import rgbfeat_scene
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    gf = np.load(os.path.join(GOLDEN, name.replace("_paths_", "_film_") + ".npz"))
    scene = rgbfeat_scene(pg, g, name, request)
    fs = rgbfeat_scene(pg, gf, name, request)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
        d.upload(fs)
        d.render()
        film = d.film()
    assert_bit_exact(L, g["L"], name)
    assert_bit_exact(film, gf["film"], name.replace("_paths_", "_film_"))


def test_integrator_scene_checks(pg):
    """pbrtgpu_scene_upload refuses what the integrator steps cannot render: a negative
    maxdepth, an unknown metadata strategy, mesh / material ids without the per-primitive id
    table.  Any maxdepth the reference reads is accepted (the RNG's full state is kept once a
    path passes 227 draws)."""
    from conftest import PACKS
    import ctypes
    pack = os.path.join(PACKS, "coverage.pack")
    with pg.Device(0) as d:
        s = pg.Scene.load(pack, xres=8, yres=8, spp=1, maxdepth=7, integrator="directlighting")
        s.flat.max_depth = -1
        with pytest.raises(RuntimeError, match="maxdepth"):
            d.upload(s)
        for md in (6, 7, 25):
            d.upload(pg.Scene.load(pack, xres=8, yres=8, spp=1, maxdepth=md, integrator="directlighting"))
        d.upload(pg.Scene.load(pack, xres=8, yres=8, spp=1, maxdepth=60))
        m = pg.Scene.load(pack, xres=8, yres=8, spp=1, integrator="metadata", strategy="mesh")
        m.flat.meta_strategy = 7
        with pytest.raises(RuntimeError, match="strategy"):
            d.upload(m)
        m.flat.meta_strategy = pg.META_STRATEGIES["material"]
        m.flat.prim_meta = None
        with pytest.raises(RuntimeError, match="prim_meta"):
            d.upload(m)
        m.flat.meta_strategy = pg.META_STRATEGIES["depth"]   # depth needs no ids
        d.upload(m)
