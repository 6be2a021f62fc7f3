"""The CPU oracle (oracle/pathtrace.c) against golden vectors produced by the reference
itself (tools/make_golden.py runs the reference harness built from the unmodified
reference sources).  This pins the oracle before it is trusted as the GPU's checker.

liboracle_libm.so calls glibc's float transcendentals -- the reference's own -- and must
match bit for bit.  liboracle.so evaluates them with include/pbrt_libmf.h, the restatement of
those glibc routines that the GPU kernels compile (pinned over every float input
by tools/libmf_check.c, tests/test_libmf.py); it must match bit for bit as well.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, PACKS


def _scene(pg, cfg, name="killeroo"):
    w, h, spp, seed, md = [int(v) for v in cfg]
    pack = {"anim": "anim-killeroos-moving.pack", "bunny": "bunny.pack", "metal": "metal.pack",
            "coverage": "coverage.pack", "imagemap": "imagemap.pack",
            "animcam": "animcam.pack", "textured": "textured.pack", "envmap": "envmap.pack", "lights": "lights.pack",
            "ortho": "ortho.pack", "heightfield": "heightfield.pack",
            "cylinder": "cylinder.pack", "anisoward": "anisoward.pack", "mappings": "mappings.pack", "checker": "checker.pack",
            "shinymetal": "shinymetal.pack", "nurbs": "nurbs.pack"}.get(name.split("_")[0],
                                                                                              "killeroo-simple.pack")
    # *_b30_*: the upstream 30-band, 400-700 nm build (b30 harness, spectrum.h.original:36-38)
    if "_b30_" in name:
        pack = pack.replace(".pack", "-b30.pack")
    return pg.Scene.load(os.path.join(PACKS, pack), xres=w, yres=h, spp=spp, maxdepth=md, seed=seed)


def exact_rate(name):
    """Fraction of paths the GPU must reproduce bit for bit: all of them (its transcendentals are
    the reference's glibc routines restated, include/pbrt_libmf.h)."""
    return 1.0


PATHS = ["killeroo_paths_64x64s4", "killeroo_paths_48x48s8_seed7_md7", "anim_paths_48x48s4", "bunny_paths_64x36s4",
         "metal_paths_48x48s4", "coverage_paths_64x48s8", "killeroo_b30_paths_48x40s4", "coverage_b30_paths_48x36s4",
         "imagemap_paths_64x48s4", "imagemap_paths_96x72s2_seed5", "animcam_paths_64x48s4", "textured_paths_64x48s4", "envmap_paths_64x48s4",
         "lights_paths_64x48s4", "ortho_paths_64x48s4", "heightfield_paths_64x48s4",
         "cylinder_paths_64x48s4", "anisoward_paths_64x48s4", "mappings_paths_64x48s4", "checker_paths_64x48s4",
         "shinymetal_paths_64x48s4", "nurbs_paths_64x48s4"]
# the configs at their real size and sample count (BASELINE.json configs 2-5; harness --keys):
# every sample of a few pixels plus random keys of the whole sample extent
KEYS = ["killeroo_keys_c2_700x700s256", "bunny_keys_c3_1920x1080s1024", "metal_keys_c4_400x400s4096",
        "anim_keys_c5_600x600s512"]
PATHS += KEYS


@pytest.fixture(scope="module")
def ora_libm(pg):
    return pg.oracle(libm_float=True)


@pytest.mark.parametrize("name", PATHS)
def test_paths_bit_exact_vs_reference(pg, ora_libm, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = _scene(pg, g["config"], name)
    L = ora_libm.trace_paths(scene, g["keys"])
    same = np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1)
    assert same.all(), "paths differing: %d / %d" % ((~same).sum(), len(same))


@pytest.mark.parametrize("name", PATHS)
def test_paths_restated_libm_bit_exact_vs_reference(pg, name):
    """The GPU's definition of the float transcendentals (include/pbrt_libmf.h) in the oracle:
    every path bit for bit the reference's."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = _scene(pg, g["config"], name)
    L = pg.oracle().trace_paths(scene, g["keys"])
    same = np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1)
    assert same.all(), "paths differing: %d / %d" % ((~same).sum(), len(same))


@pytest.mark.parametrize("name", ["killeroo_film_96x72s16", "anim_film_40x40s8", "bunny_film_48x27s8",
                                  "metal_film_40x40s8", "coverage_film_64x48s8", "killeroo_b30_film_40x32s8",
                                  "coverage_b30_film_40x30s4", "imagemap_film_64x48s8",
                                  "animcam_film_64x48s4", "textured_film_64x48s8", "envmap_film_64x48s8",
                                  "lights_film_64x48s8", "ortho_film_64x48s4", "heightfield_film_64x48s4",
                                  "cylinder_film_64x48s4", "anisoward_film_64x48s4", "mappings_film_64x48s4", "checker_film_64x48s4",
                                  "shinymetal_film_64x48s4", "nurbs_film_64x48s4"])
def test_film_bit_exact_vs_reference(pg, ora_libm, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = _scene(pg, g["config"], name)
    film, st = ora_libm.render(scene, threads=8)
    if name.startswith("killeroo_film"):
        assert st[2] > 0, "fixture should contain samples landing on neighbour pixels"
    assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))


def test_mt19937_known_answers(pg):
    g = np.load(os.path.join(GOLDEN, "mt19937_kat.npz"))
    o = pg.oracle()
    for seed, out in zip(g["seeds"], g["out"]):
        assert np.array_equal(o.mt_first(int(seed), 64), out)
    # the canonical MT19937 check value (seed 5489, 10000th output)
    assert int(o.mt_first(5489, 10000)[-1]) == 4123659995


@pytest.mark.parametrize("bands", [32, 60, 30])
def test_host_fromrgb_bit_exact(pg, bands):
    g = np.load(os.path.join(GOLDEN, "fromrgb_%d.npz" % bands))
    for rgb, refl, illum in zip(g["rgb"], g["refl"], g["illum"]):
        assert np.array_equal(pg.spectrum_from_rgb(rgb, bands).view(np.int32), refl.view(np.int32))
        assert np.array_equal(pg.spectrum_from_rgb(rgb, bands, illuminant=True).view(np.int32), illum.view(np.int32))


def test_metal_scene_contents(pg):
    """C4 pack: 60 bands, the Au metal, the textured substrate floor, the environment light."""
    from conftest import PACKS
    s = pg.Scene.load(os.path.join(PACKS, "metal.pack"), xres=16, yres=16, spp=1)
    assert s.bands == 60 and s.flat.n_textures >= 3 and s.flat.n_lights == 1
    import ctypes
    assert ctypes.cast(s.flat.lights, ctypes.POINTER(ctypes.c_int32))[0] == 2   # PBRTGPU_LIGHT_INFINITE


@pytest.mark.parametrize("name", ["merl_paths_64x48s8", "merl_film_64x48s8"])
def test_regular_halfangle_brdf_bit_exact_vs_reference(pg, ora_libm, merl_dir, name):
    """RegularHalfangleBRDF (reflection.cpp:267-300) from a MERL-format table loaded as
    measured.cpp:131-175 loads it, and a measured material whose file is missing (no BxDF):
    the oracle against the reference harness, bit for bit."""
    from conftest import merl_scene
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = merl_scene(pg, merl_dir, g["config"])
    assert scene.flat.n_merl_floats == 3 * 90 * 90 * 180
    if "paths" in name:
        L = ora_libm.trace_paths(scene, g["keys"])
        same = np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1)
        assert same.all(), "paths differing: %d / %d" % ((~same).sum(), len(same))
    else:
        film, _ = ora_libm.render(scene, threads=8)
        assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))


DL = ["checker_dl_%s_48x36s4", "mappings_dl_%s_48x36s4", "shinymetal_dl_%s_48x36s4", "anisoward_dl_%s_48x36s4", "cylinder_dl_%s_48x36s4", "ortho_dl_%s_48x36s4", "lights_dl_%s_48x36s4", "textured_dl_%s_48x36s4", "envmap_dl_%s_48x36s4", "killeroo_dl_%s_48x40s4", "bunny_dl_%s_48x27s4", "anim_dl_%s_40x40s4", "coverage_dl_%s_64x48s4",
      "coverage_dlone_%s_64x48s4"]


def dl_scene(pg, g, name):
    """The pack of a DirectLightingIntegrator fixture, rendered with the integrator the scene
    files name (packs record "path", the configs' override)."""
    w, h, spp, seed, md = [int(v) for v in g["config"]]
    pack = {"anim": "anim-killeroos-moving.pack", "bunny": "bunny.pack", "coverage": "coverage.pack",
            "textured": "textured.pack", "envmap": "envmap.pack", "lights": "lights.pack",
            "ortho": "ortho.pack", "heightfield": "heightfield.pack",
            "cylinder": "cylinder.pack", "anisoward": "anisoward.pack", "mappings": "mappings.pack", "checker": "checker.pack",
            "shinymetal": "shinymetal.pack", "nurbs": "nurbs.pack"}.get(
        name.split("_")[0], "killeroo-simple.pack")
    return pg.Scene.load(os.path.join(PACKS, pack), xres=w, yres=h, spp=spp, maxdepth=md, seed=seed,
                         integrator="directlighting", strategy="one" if "_dlone_" in name else "all")


@pytest.mark.parametrize("name", [d % "paths" for d in DL])
def test_direct_lighting_paths_bit_exact_vs_reference(pg, ora_libm, name):
    """DirectLightingIntegrator (directlighting.cpp:73-109; UniformSampleAllLights /
    UniformSampleOneLight, integrator.cpp:39-106; SpecularReflect / SpecularTransmit with ray
    differentials, integrator.cpp:169-250): the oracle against the reference harness."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = dl_scene(pg, g, name)
    assert scene.flat.integrator == pg.INTEGRATORS["directlighting"]
    L = ora_libm.trace_paths(scene, g["keys"])
    same = np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1)
    assert same.all(), "paths differing: %d / %d" % ((~same).sum(), len(same))


@pytest.mark.parametrize("name", [d % "film" for d in DL])
def test_direct_lighting_film_bit_exact_vs_reference(pg, ora_libm, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    film, _ = ora_libm.render(dl_scene(pg, g, name), threads=8)
    assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))


META = ["metadata_material_%s_48x36s4", "metadata_mesh_%s_48x36s4", "metadata_depth_%s_48x36s4",
        "killeroo_meta_mesh_%s_40x32s2", "anim_meta_mesh_%s_40x32s2", "bunny_meta_depth_%s_40x32s2",
        "heightfield_meta_mesh_%s_48x36s2", "nurbs_meta_mesh_%s_48x36s2"]


def meta_scene(pg, g, name):
    """The scene of a MetadataIntegrator fixture: tests/scenes/metadata.pbrt itself, or a config
    scene's pack rendered with integrator "metadata" and the fixture's strategy."""
    w, h, spp, seed, md = [int(v) for v in g["config"]]
    st = "mesh" if "_mesh_" in name else "material" if "_material_" in name else "depth"
    if name.startswith("metadata_"):
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes", "metadata.pbrt")
    else:
        path = os.path.join(PACKS, {"anim": "anim-killeroos-moving.pack", "bunny": "bunny.pack",
                                    "heightfield": "heightfield.pack", "nurbs": "nurbs.pack"}.get(
            name.split("_")[0], "killeroo-simple.pack"))
    return pg.Scene.load(path, xres=w, yres=h, spp=spp, seed=seed, integrator="metadata", strategy=st)


@pytest.mark.parametrize("name", [m % "paths" for m in META])
def test_metadata_paths_bit_exact_vs_reference(pg, ora_libm, name):
    """MetadataIntegrator (metadata.cpp:41-98): Spectrum(primitiveId / materialId / depth) of
    the first hit, the ids replayed from the reference's Primitive / Material constructor
    counters by the front end; the oracle against the reference harness, bit for bit."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = meta_scene(pg, g, name)
    L = ora_libm.trace_paths(scene, g["keys"])
    assert np.array_equal(L.view(np.int32), g["L"].view(np.int32))


@pytest.mark.parametrize("name", [m % "film" for m in META])
def test_metadata_film_bit_exact_vs_reference(pg, ora_libm, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    film, _ = ora_libm.render(meta_scene(pg, g, name), threads=8)
    assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))


SPEC = ["killeroo_spec32_%s_40x32s4", "coverage_spec3_%s_48x36s4", "coverage_specsampler8_%s_48x36s8",
        "killeroo_spec5_dl_%s_32x24s2", "killeroo_b30_spec5_%s_32x24s4", "coverage_b30_specsampler6_%s_40x30s8"]


def spec_scene(pg, g, name):
    """The scene of a SpectralRenderer fixture: the pack (or tests/scenes/coverage.pbrt's pack)
    rendered with renderer "spectral", the fixture's nWaveBands and samplingMethod (and the
    DirectLightingIntegrator for the _dl fixture)."""
    w, h, spp, seed, md = [int(v) for v in g["config"]]
    pack = "coverage.pack" if name.startswith("coverage") else "killeroo-simple.pack"
    if "_b30_" in name:   # the 30-band build: wave bands over 400-700 nm
        pack = pack.replace(".pack", "-b30.pack")
    tok = [t for t in name.split("_") if t.startswith("spec")][0]
    nwb = int(tok.replace("specsampler", "").replace("spec", ""))
    return pg.Scene.load(os.path.join(PACKS, pack), xres=w, yres=h, spp=spp, maxdepth=md, seed=seed,
                         integrator="directlighting" if "_dl_" in name else "path", renderer="spectral", wave_bands=nwb,
                         sampling="sampler" if "specsampler" in name else "single")


@pytest.mark.parametrize("name", [m % "paths" for m in SPEC])
def test_spectral_renderer_paths_bit_exact_vs_reference(pg, ora_libm, name):
    """SpectralRenderer (spectralrenderer.cpp:98-190): per camera sample and wave band a path
    whose radiance at the band's wavelength (Spectrum::GetValueAtWavelength, spectrum.h:384-405)
    fills the band's indices; the oracle against the reference harness, bit for bit."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = spec_scene(pg, g, name)
    assert scene.flat.renderer == pg.RENDERERS["spectral"]
    L = ora_libm.trace_paths(scene, g["keys"])
    same = np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1)
    assert same.all(), "samples differing: %d / %d" % ((~same).sum(), len(same))


@pytest.mark.parametrize("name", [m % "film" for m in SPEC])
def test_spectral_renderer_film_bit_exact_vs_reference(pg, ora_libm, name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    film, _ = ora_libm.render(spec_scene(pg, g, name), threads=8)
    assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))


RGB = ["killeroo_rgb_paths_48x40s4", "killeroo_rgb_film_40x32s8", "killeroo_rgb_keys_c1_400x400s64"]


def rgb_scene(pg, g):
    """C1: killeroo-simple in the reference's RGB build (Spectrum = RGBSpectrum, pbrt.h:144), from
    its 3-channel pack."""
    w, h, spp, seed, md = [int(v) for v in g["config"]]
    return pg.Scene.load(os.path.join(PACKS, "killeroo-simple-rgb.pack"), xres=w, yres=h, spp=spp, maxdepth=md,
                         seed=seed)


@pytest.mark.parametrize("name", RGB)
def test_rgb_build_bit_exact_vs_reference(pg, ora_libm, name):
    """C1 (BASELINE configs[0]): the RGBSpectrum build of the reference harness (oracle/ref
    BANDS=rgb) against the oracle with 3 channels -- FromRGB keeps the triple, y() weighs it
    with RGBSpectrum's YWeight -- per path (including keys at C1's 400x400 at 64 spp) and film."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = rgb_scene(pg, g)
    assert scene.bands == 3
    if "film" in name:
        film, _ = ora_libm.render(scene, threads=8)
        assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))
    else:
        L = ora_libm.trace_paths(scene, g["keys"])
        assert np.array_equal(L.view(np.int32), g["L"].view(np.int32))


# the RGB build on the feature scenes (tools/make_golden.py --only rgbfeat): image textures and
# normal maps, textured parameters with sampled-spectrum operands (RGBSpectrum::FromSampled), the
# image-based environment light, the coverage scene (SPD metals, every light type), MERL tables
RGBFEAT = ["%s_rgb_paths_64x48s4" % s for s in ("imagemap", "textured", "envmap", "coverage", "merl", "lights")] + \
          ["%s_rgb_film_64x48s4" % s for s in ("imagemap", "textured", "envmap", "coverage", "merl", "lights")] + \
          ["envmap_rgb_dl_paths_48x36s4", "envmap_rgb_dl_film_48x36s4", "coverage_rgb_dl_paths_48x36s4",
           "coverage_rgb_dl_film_48x36s4"]


def rgbfeat_scene(pg, g, name, request):
    """tests/scenes/<stem>.pbrt parsed for the RGB build (bands = 3; merl.pbrt next to its table),
    DirectLighting for the _dl_ fixtures"""
    w, h, spp, seed, md = [int(v) for v in g["config"]]
    stem = name.split("_")[0]
    if stem == "merl":
        path = os.path.join(request.getfixturevalue("merl_dir"), "merl.pbrt")
    else:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes", stem + ".pbrt")
    kw = {"integrator": "directlighting", "strategy": "all"} if "_dl_" in name else {}
    return pg.Scene.load(path, xres=w, yres=h, spp=spp, maxdepth=md, seed=seed, bands=3, **kw)


@pytest.mark.parametrize("name", RGBFEAT)
def test_rgb_build_features_bit_exact_vs_reference(pg, ora_libm, name, request):
    """The RGBSpectrum build beyond C1's scene: FromRGB is the triple for image-texture lookups,
    the environment map's radiance and MERL texels, FromSampled integrates the 1 nm CIE functions
    (spectrum.h:493-516); the oracle against the brgb harness, bit for bit."""
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = rgbfeat_scene(pg, g, name, request)
    assert scene.bands == 3
    if "_film_" in name:
        film, _ = ora_libm.render(scene, threads=8)
        assert np.array_equal(film.view(np.int32), g["film"].view(np.int32))
    else:
        L = ora_libm.trace_paths(scene, g["keys"])
        assert np.any(L != 0)
        same = np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1)
        assert same.all(), "paths differing: %d / %d" % ((~same).sum(), len(same))
