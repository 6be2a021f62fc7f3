"""Generate tests/golden/* from the reference harness (oracle/_ref, built from the unmodified
reference sources by oracle/ref/Makefile).  Runs only in the build container, where
/root/reference exists; the fixtures it writes are committed and are all the GPU box and the
CPU test suite need.

Fixtures (numpy .npz, inputs + expected outputs only):
  killeroo_paths_64x64s4.npz      per-path radiance of every 5th path (x, y, s keys) of
                                  killeroo-simple at 64x64, 4 spp, seed 0, maxdepth 5
  killeroo_paths_48x48s8_seed7_md7.npz   every 3rd path, 8 spp, seed 7, maxdepth 7 (MT19937 draws)
  killeroo_film_96x72s16.npz      raw film sums [72][96][32] at 96x72, 16 spp (includes 3 samples
                                  that land on neighbouring pixels)
  anim_paths_48x48s4.npz, anim_film_40x40s8.npz   the motion-blur scene (C5): animated
                                  TransformedPrimitives over nested BVHs
  bunny_paths_64x36s4.npz, bunny_film_48x27s8.npz   C3: measured BRDF (mystique, kd-tree
                                  lookups), point light, disk area light
  mt19937_kat.npz                 first 64 outputs of RNG(seed) for 6 seeds
  fromrgb_32.npz                  SampledSpectrum::FromRGB (reflectance and illuminant) for 14
                                  RGB triples, 32 bands 395-715 nm
  coverage_paths_64x48s8.npz, coverage_film_64x48s8.npz   tests/scenes/coverage.pbrt (this
                                  repository's feature-coverage scene): glass, mirror, Oren-Nayar,
                                  copper metal with textured bump, scaled/trilinear/black-wrap
                                  textures, disk + point + environment lights, maxdepth 6
  metal_paths_48x48s4.npz, metal_film_40x40s8.npz, fromrgb_60.npz   C4, 60-band build (b60
                                  harness): Au metal (FresnelConductor from SPD files), substrate
                                  floor with imagemap Kd + scaled imagemap bump (1x1 fallback
                                  texels, EWA filtering with camera ray differentials), infinite
                                  light (one-texel environment map)
  <scene>_keys_<cfg>_*.npz         per-path radiance at the configs' REAL size and sample count
                                  (C2 killeroo 700x700@256, C3 bunny 1920x1080@1024, C4 metal
                                  400x400@4096 60 bands, C5 anim 600x600@512): every sample of a
                                  few pixels (all of the sampler's permutation masks at that spp)
                                  plus 2048 random (x, y, s) keys of the sample extent (--keys)
  merl_paths_64x48s8.npz, merl_film_64x48s8.npz   tests/scenes/merl.pbrt: RegularHalfangleBRDF
                                  (measured.cpp:131-175, reflection.cpp:267-300) from the synthetic
                                  MERL table of tools/make_merl.py, plus a measured material whose
                                  .merl file is missing (no BxDF)
  *_dl_paths_*, *_dl_film_*, coverage_dlone_*   DirectLightingIntegrator (directlighting.cpp, with
                                  UniformSampleAll/OneLight and the specular recursion of
                                  integrator.cpp:169-250): killeroo (strategy all, light nsamples 8),
                                  bunny, anim, and the coverage scene (mirror / glass recursion,
                                  textures) with strategies all and one
  metadata_*, *_meta_*            MetadataIntegrator (integrators/metadata.cpp) with strategies
                                  material / mesh / depth: tests/scenes/metadata.pbrt (named and
                                  per-shape materials, mesh, subdivision, quadric and animated
                                  primitives), killeroo and anim (mesh ids), bunny (depth)
  killeroo_dat_40x32s4.npz        the raw film of the restatement film AND the .dat the
                                  reference's own SpectralImageNoCameraFilm wrote for the same
                                  samples (--refdat): pins AddSample and the WriteImage payload
  *_b30_*, fromrgb_30.npz         the upstream 30-band build (b30 harness, 400-700 nm)
  imagemap_*                      tests/scenes/imagemap.pbrt: TGA / PFM image maps decoded by the
                                  reference's imageio.cpp into MIPMap pyramids (mipmap.h): EWA
                                  over several levels, trilinear, noFiltering, repeat / clamp / black,
                                  normal maps (image, scaled, constant)
  animcam_*                       tests/scenes/animcam.pbrt: an animated camera (AnimatedTransform
                                  CameraToWorld interpolated per ray, camera.cpp:84-103)
  textured_*                      tests/scenes/textured.pbrt: every material parameter as a texture
                                  (two textured spectra per material, textured roughness / sigma /
                                  index, metal eta / k unclamped), path and DirectLighting
  envmap_*                        tests/scenes/envmap.pbrt: an image-based infinite light (decoded PFM
                                  lat-long map: radiance MIPMap, Distribution2D sampling and pdf)
  nurbs_*                         tests/scenes/nurbs.pbrt: NURBS patches refined into meshes, path and
                                  metadata mesh ids
  mappings_*                      tests/scenes/mappings.pbrt: spherical, cylindrical and planar 2D
                                  texture mappings (image textures and bump maps), path and
                                  DirectLighting
  checker_*                       tests/scenes/checker.pbrt: Checkerboard2DTexture (closed-form box
                                  filter and point sampled, constant / image operands, uv, planar and
                                  spherical mappings, float checkerboards as bump and roughness),
                                  path and DirectLighting
  shinymetal_*                    tests/scenes/shinymetal.pbrt: shinymetal (conductor microfacet and
                                  mirror lobes), path and DirectLighting
  anisoward_*                     tests/scenes/anisoward.pbrt: the fork's anisotropic Ward material
                                  (anisoward.cpp, AnisoWardBrdf.cpp), path and DirectLighting
  cylinder_*                      tests/scenes/cylinder.pbrt: cylinders (phimax, inside / outside hits,
                                  textured, reversed, area light), path and DirectLighting
  heightfield_*                   tests/scenes/heightfield.pbrt: heightfield shapes (terrain, area
                                  light), path and metadata (mesh ids)
  ortho_*                         tests/scenes/ortho.pbrt: the orthographic camera (screen window,
                                  thin lens, shutter, ray differentials), path and DirectLighting
  lights_*                        tests/scenes/lights.pbrt: spot lights (falloff band, transformed
                                  frames) and a distant light beside an area light (path, DL, RGB)
  <scene>_rgb_*                   the RGB build (brgb harness, Spectrum = RGBSpectrum) on imagemap,
                                  textured, envmap, coverage and merl: image textures and normal
                                  maps, RGBSpectrum::FromSampled (SPD metals, sampled operands), the
                                  environment map, MERL tables; DirectLighting on envmap / coverage
  coverage_gpupath_dat_40x32s4.npz   the .dat the reference's own spectral film writes for
                                  tests/scenes/coverage.pbrt (--refdat, the scene's integrator): the
                                  end-to-end check of Renderer "gpupath" (tests/test_binding_gpu.py)
  <scene>_window_<cfg>_*.npz      film crops at the configs' REAL size and sample count: every
                                  sample of a one-pixel-larger window (--window), so each cropped
                                  pixel holds all of its contributions (incl. exact-boundary samples
                                  of its neighbours, spectralImage.cpp:77-152); C2 at the sphere
                                  light's edge and at a killeroo silhouette, C3-C5 at an edge each
Usage: python tools/make_golden.py [--only keys|dat|merl|dl|meta|spec|rgb|rgbfeat|mappings|checker|lights|ortho|heightfield|cylinder|anisoward|shinymetal|nurbs|b30|window|imagemap|animcam|gpupath|textured|envmap]
       (after `make -C oracle ref`, `ref60`, `ref30` and `refrgb`)
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "b32", "pbrt_ref_harness")
HARNESS60 = os.path.join(ROOT, "oracle", "_ref", "b60", "pbrt_ref_harness")   # make -C oracle ref60
HARNESSRGB = os.path.join(ROOT, "oracle", "_ref", "brgb", "pbrt_ref_harness")  # make -C oracle refrgb
HARNESS30 = os.path.join(ROOT, "oracle", "_ref", "b30", "pbrt_ref_harness")    # make -C oracle ref30
SCENES = "/root/reference/scenes"
OUT = os.path.join(ROOT, "tests", "golden")


def run(args, bands=32):
    exe = {60: HARNESS60, 30: HARNESS30, 3: HARNESSRGB}.get(bands, HARNESS)
    subprocess.run([exe] + args, check=True, cwd=SCENES)


def read_paths(fn):
    raw = np.fromfile(fn, dtype=np.int32)
    nb, spp, seed = raw[0], raw[1], raw[2]
    rec = raw[4:].reshape(-1, 3 + nb)
    return rec[:, :3].copy(), rec[:, 3:].copy().view(np.float32), int(spp), int(seed)


def paths_fixture(name, res, spp, seed, maxdepth, every, tmp, scene="killeroo-simple.pbrt", bands=32, extra=()):
    fn = os.path.join(tmp, name + ".bin")
    run([os.path.join(SCENES, scene), "--res", str(res[0]), str(res[1]), "--spp", str(spp), "--seed", str(seed), "--maxdepth",
         str(maxdepth), "--paths", fn, "--path-every", str(every)] + list(extra), bands)
    keys, L, _, _ = read_paths(fn)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), keys=keys, L=L,
                        config=np.array([res[0], res[1], spp, seed, maxdepth], np.int32))
    print(name, keys.shape)


def film_fixture(name, res, spp, seed, maxdepth, tmp, scene="killeroo-simple.pbrt", bands=32, extra=()):
    fn = os.path.join(tmp, name + ".f32")
    run([os.path.join(SCENES, scene), "--res", str(res[0]), str(res[1]), "--spp", str(spp), "--seed", str(seed), "--maxdepth",
         str(maxdepth), "--raw", fn] + list(extra), bands)
    raw = np.fromfile(fn, dtype=np.int32)
    W, H, N = raw[:3]
    film = raw[3:].view(np.float32).reshape(H, W, N)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), film=film,
                        config=np.array([res[0], res[1], spp, seed, maxdepth], np.int32))
    print(name, film.shape)


# (name, scene file, pack, W, H, spp, bands, key seed): BASELINE.json configs 2-5 at full size
KEY_CONFIGS = [("killeroo_keys_c2_700x700s256", "killeroo-simple.pbrt", 700, 700, 256, 32, 2),
               ("bunny_keys_c3_1920x1080s1024", "bunny.pbrt", 1920, 1080, 1024, 32, 3),
               ("metal_keys_c4_400x400s4096", "metal.pbrt", 400, 400, 4096, 60, 4),
               ("anim_keys_c5_600x600s512", "anim-killeroos-moving.pbrt", 600, 600, 512, 32, 5)]


def config_keys(W, H, spp, seed, n_random=2048):
    """Every sample of max(1, 4096 // spp) random pixels, then n_random random keys, over the
    box filter's sample extent [0, W + 1) x [0, H + 1) (spectralImage.cpp:176-185)."""
    rng = np.random.RandomState(seed)
    npx = max(1, 4096 // spp)
    px = np.stack([rng.randint(0, W + 1, npx), rng.randint(0, H + 1, npx)], 1)
    full = np.array([(x, y, s) for x, y in px for s in range(spp)], np.int32).reshape(-1, 3)
    rnd = np.stack([rng.randint(0, W + 1, n_random), rng.randint(0, H + 1, n_random), rng.randint(0, spp, n_random)], 1)
    return np.concatenate([full, rnd.astype(np.int32)])


def rgb_fixtures(tmp):
    """C1: the reference's RGB build (Spectrum = RGBSpectrum) on killeroo-simple -- per-path RGB
    radiance, a film, and keys at C1's real size (400x400 at 64 spp)."""
    paths_fixture("killeroo_rgb_paths_48x40s4", (48, 40), 4, 0, 5, 1, tmp, bands=3)
    film_fixture("killeroo_rgb_film_40x32s8", (40, 32), 8, 0, 5, tmp, bands=3)
    keys_fixture("killeroo_rgb_keys_c1_400x400s64", "killeroo-simple.pbrt", 400, 400, 64, 3, 1, tmp)


def rgbfeat_fixtures(tmp):
    """The RGB build (Spectrum = RGBSpectrum) on the feature scenes: decoded image textures and
    normal / bump maps, textured material parameters (sampled-spectrum operands through
    RGBSpectrum::FromSampled), the image-based environment light, the coverage scene (SPD metals,
    every light type), a RegularHalfangle MERL table; path integrator and DirectLighting"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_merl
    sd = os.path.join(ROOT, "tests", "scenes")
    make_merl.write(os.path.join(sd, "synthetic.merl"))   # git-ignored, regenerated here
    for stem, scene, md in (("imagemap", "imagemap.pbrt", 3), ("textured", "textured.pbrt", 5),
                            ("envmap", "envmap.pbrt", 5), ("coverage", "coverage.pbrt", 6), ("merl", "merl.pbrt", 5)):
        sc = os.path.join(sd, scene)
        paths_fixture("%s_rgb_paths_64x48s4" % stem, (64, 48), 4, 0, md, 1, tmp, scene=sc, bands=3)
        film_fixture("%s_rgb_film_64x48s4" % stem, (64, 48), 4, 0, md, tmp, scene=sc, bands=3)
    for stem, scene in (("envmap", "envmap.pbrt"), ("coverage", "coverage.pbrt")):
        sc = os.path.join(sd, scene)
        ex = ("--surf", "directlighting", "--dl-strategy", "all")
        paths_fixture("%s_rgb_dl_paths_48x36s4" % stem, (48, 36), 4, 0, 5, 1, tmp, scene=sc, bands=3, extra=ex)
        film_fixture("%s_rgb_dl_film_48x36s4" % stem, (48, 36), 4, 0, 5, tmp, scene=sc, bands=3, extra=ex)


def spectra_fixture(bands, tmp):
    """SampledSpectrum::FromRGB (reflectance and illuminant) of the harness's RGB triples."""
    fn = os.path.join(tmp, "spec%d.bin" % bands)
    run(["-", "--spectra", fn], bands)
    raw = np.fromfile(fn, dtype=np.int32)
    n = raw[0]
    rec = raw[1:].reshape(n, 3 + 2 * bands).view(np.float32)
    np.savez_compressed(os.path.join(OUT, "fromrgb_%d.npz" % bands), rgb=rec[:, :3].copy(), refl=rec[:, 3:3 + bands].copy(),
                        illum=rec[:, 3 + bands:].copy())


def b30_fixtures(tmp):
    """The upstream 30-band build (400-700 nm, spectrum.h.original:36-38; BASELINE's literal
    "30 bands"): killeroo (C2's scene) and the coverage scene (SPD metals, textures, every light
    type), per-path radiance and film, and FromRGB."""
    paths_fixture("killeroo_b30_paths_48x40s4", (48, 40), 4, 0, 5, 2, tmp, bands=30)
    film_fixture("killeroo_b30_film_40x32s8", (40, 32), 8, 0, 5, tmp, bands=30)
    cov = os.path.join(ROOT, "tests", "scenes", "coverage.pbrt")
    paths_fixture("coverage_b30_paths_48x36s4", (48, 36), 4, 0, 6, 1, tmp, scene=cov, bands=30)
    film_fixture("coverage_b30_film_40x30s4", (40, 30), 4, 0, 6, tmp, scene=cov, bands=30)
    spectra_fixture(30, tmp)
    # the SpectralRenderer at 30 bands: wave-band wavelengths from 400 / 700 nm
    for stem, scene, res, spp, nwb, method, md in (("killeroo_b30_spec5", "killeroo-simple.pbrt", (32, 24), 4, 5, "single", 5),
                                                   ("coverage_b30_specsampler6", cov, (40, 30), 8, 6, "sampler", 6)):
        ex = ("--spectral", str(nwb), method, "--surf", "path")
        tag = "%dx%ds%d" % (res[0], res[1], spp)
        paths_fixture("%s_paths_%s" % (stem, tag), res, spp, 0, md, 1, tmp, scene=scene, bands=30, extra=ex)
        film_fixture("%s_film_%s" % (stem, tag), res, spp, 0, md, tmp, scene=scene, bands=30, extra=ex)


def keys_fixture(name, scene, W, H, spp, bands, kseed, tmp):
    keys = config_keys(W, H, spp, kseed)
    kf = os.path.join(tmp, name + ".keys")
    keys.astype(np.int32).tofile(kf)
    fn = os.path.join(tmp, name + ".bin")
    run([os.path.join(SCENES, scene), "--res", str(W), str(H), "--spp", str(spp), "--seed", "0", "--maxdepth", "5",
         "--keys", kf, "--paths", fn], bands)
    k2, L, _, _ = read_paths(fn)
    assert np.array_equal(k2, keys)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), keys=keys, L=L, config=np.array([W, H, spp, 0, 5], np.int32))
    print(name, keys.shape)


# (name, scene file, W, H, spp, bands, film-pixel window x0, y0, w, h): tile-aligned (16 x 16)
# crops of BASELINE.json configs 2-5 at full resolution and spp
WINDOW_CONFIGS = [("killeroo_window_c2_light_700x700s256", "killeroo-simple.pbrt", 700, 700, 256, 32, 64, 16, 48, 48),
                  ("killeroo_window_c2_edge_700x700s256", "killeroo-simple.pbrt", 700, 700, 256, 32, 96, 288, 48, 48),
                  ("bunny_window_c3_1920x1080s1024", "bunny.pbrt", 1920, 1080, 1024, 32, 1216, 832, 32, 32),
                  ("metal_window_c4_400x400s4096", "metal.pbrt", 400, 400, 4096, 60, 96, 112, 32, 32),
                  ("anim_window_c5_600x600s512", "anim-killeroos-moving.pbrt", 600, 600, 512, 32, 112, 240, 32, 32)]


def window_fixture(name, scene, W, H, spp, bands, x0, y0, w, h, tmp):
    """Film pixels [x0, x0 + w) x [y0, y0 + h) of the full-size render.  Film pixel x receives
    samples of sample pixels x - 1, x, x + 1 only (the box filter's footprint, two pixels wide at
    an exact boundary), so the harness traces the sample window one pixel larger on each side."""
    fn = os.path.join(tmp, name + ".f32")
    run([os.path.join(SCENES, scene), "--res", str(W), str(H), "--spp", str(spp), "--seed", "0", "--maxdepth", "5",
         "--window", str(x0 - 1), str(x0 + w + 1), str(y0 - 1), str(y0 + h + 1), "--raw", fn], bands)
    raw = np.fromfile(fn, dtype=np.int32)
    FW, FH, N = raw[:3]
    film = raw[3:].view(np.float32).reshape(FH, FW, N)[y0:y0 + h, x0:x0 + w].copy()
    np.savez_compressed(os.path.join(OUT, name + ".npz"), film=film, window=np.array([x0, y0, w, h], np.int32),
                        config=np.array([W, H, spp, 0, 5], np.int32))
    print(name, film.shape)


def dat_fixture(name, res, spp, tmp, scene="killeroo-simple.pbrt"):
    """The restatement film (--raw) and the reference film's .dat (--refdat) of one render."""
    raw, dat = os.path.join(tmp, name + ".f32"), os.path.join(tmp, name + ".dat")
    run([os.path.join(SCENES, scene), "--res", str(res[0]), str(res[1]), "--spp", str(spp), "--seed", "0", "--maxdepth",
         "5", "--raw", raw, "--refdat", dat])
    r = np.fromfile(raw, dtype=np.int32)
    W, H, N = r[:3]
    film = r[3:].view(np.float32).reshape(H, W, N)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), film=film, dat=np.fromfile(dat, dtype=np.uint8),
                        config=np.array([res[0], res[1], spp, 0, 5], np.int32))
    print(name, film.shape, os.path.getsize(dat))


# DirectLightingIntegrator (the integrator the packaged scene files name): (fixture stem, scene,
# res, spp, maxdepth, path stride, harness extra args).  Python loads the matching pack with
# integrator="directlighting" (and strategy="one" for the dlone fixtures).
DL_FIXTURES = [
    ("killeroo_dl", "killeroo-simple.pbrt", (48, 40), 4, 5, 2, ()),            # strategy all, nsamples 8
    ("bunny_dl", "bunny.pbrt", (48, 27), 4, 5, 2, ()),                        # point + disk (nsamples 4)
    ("anim_dl", "anim-killeroos-moving.pbrt", (40, 40), 4, 5, 2, ()),         # instances, motion blur
    ("coverage_dl", "COVERAGE", (64, 48), 4, 6, 1, ()),                       # mirror / glass recursion, textures
    ("coverage_dlone", "COVERAGE", (64, 48), 4, 6, 1, ("--dl-strategy", "one")),
]


def dl_fixtures(tmp):
    for stem, scene, res, spp, md, every, extra in DL_FIXTURES:
        if scene == "COVERAGE":
            scene = os.path.join(ROOT, "tests", "scenes", "coverage.pbrt")
        ex = ("--surf", "directlighting") + tuple(extra)
        tag = "%dx%ds%d" % (res[0], res[1], spp)
        paths_fixture("%s_paths_%s" % (stem, tag), res, spp, 0, md, every, tmp, scene=scene, extra=ex)
        film_fixture("%s_film_%s" % (stem, tag), res, spp, 0, md, tmp, scene=scene, extra=ex)


# MetadataIntegrator (integrators/metadata.cpp): (fixture stem, scene, res, spp, strategy, stride).
# Python loads tests/scenes/metadata.pbrt directly and the config scenes from their packs with
# integrator="metadata" and the strategy.
META_FIXTURES = [
    ("metadata_material", "METADATA", (48, 36), 4, "material", 1),   # named + per-shape materials
    ("metadata_mesh", "METADATA", (48, 36), 4, "mesh", 1),           # mesh / subdivision / quadric / animated ids
    ("metadata_depth", "METADATA", (48, 36), 4, "depth", 1),
    ("killeroo_meta_mesh", "killeroo-simple.pbrt", (40, 32), 2, "mesh", 1),
    ("anim_meta_mesh", "anim-killeroos-moving.pbrt", (40, 32), 2, "mesh", 1),
    ("bunny_meta_depth", "bunny.pbrt", (40, 32), 2, "depth", 1),
]


def meta_fixtures(tmp):
    for stem, scene, res, spp, st, every in META_FIXTURES:
        if scene == "METADATA":
            scene = os.path.join(ROOT, "tests", "scenes", "metadata.pbrt")
        ex = ("--surf", "metadata", "--meta-strategy", st)
        tag = "%dx%ds%d" % (res[0], res[1], spp)
        paths_fixture("%s_paths_%s" % (stem, tag), res, spp, 0, 5, every, tmp, scene=scene, extra=ex)
        film_fixture("%s_film_%s" % (stem, tag), res, spp, 0, 5, tmp, scene=scene, extra=ex)


# SpectralRenderer (renderers/spectralrenderer.cpp): (fixture stem, scene, res, spp, nWaveBands,
# samplingMethod, surface integrator, path stride).  Python loads the packs / coverage scene with
# renderer="spectral", wave_bands and sampling (and the integrator).
SPEC_FIXTURES = [
    ("killeroo_spec32", "killeroo-simple.pbrt", (40, 32), 4, 32, "single", "path", 1),   # the defaults
    ("coverage_spec3", "COVERAGE", (48, 36), 4, 3, "single", "path", 1),
    ("coverage_specsampler8", "COVERAGE", (48, 36), 8, 8, "sampler", "path", 1),
    ("killeroo_spec5_dl", "killeroo-simple.pbrt", (32, 24), 2, 5, "single", "directlighting", 1),
]


def spec_fixtures(tmp):
    for stem, scene, res, spp, nwb, method, surf, every in SPEC_FIXTURES:
        if scene == "COVERAGE":
            scene = os.path.join(ROOT, "tests", "scenes", "coverage.pbrt")
        ex = ("--spectral", str(nwb), method, "--surf", surf)
        md = 6 if "coverage" in stem else 5
        tag = "%dx%ds%d" % (res[0], res[1], spp)
        paths_fixture("%s_paths_%s" % (stem, tag), res, spp, 0, md, every, tmp, scene=scene, extra=ex)
        film_fixture("%s_film_%s" % (stem, tag), res, spp, 0, md, tmp, scene=scene, extra=ex)


def merl_fixtures(tmp):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_merl
    merl = os.path.join(ROOT, "tests", "scenes", "synthetic.merl")   # git-ignored, regenerated here
    make_merl.write(merl)
    scene = os.path.join(ROOT, "tests", "scenes", "merl.pbrt")
    paths_fixture("merl_paths_64x48s8", (64, 48), 8, 0, 5, 2, tmp, scene=scene)
    film_fixture("merl_film_64x48s8", (64, 48), 8, 0, 5, tmp, scene=scene)


def imagemap_fixtures(tmp):
    """tests/scenes/imagemap.pbrt: decoded TGA / PFM image maps in MIPMap pyramids (EWA over
    several levels, trilinear, noFiltering, the three wrap modes, float and spectrum textures)"""
    sc = os.path.join(ROOT, "tests", "scenes", "imagemap.pbrt")
    paths_fixture("imagemap_paths_64x48s4", (64, 48), 4, 0, 3, 1, tmp, scene=sc)
    film_fixture("imagemap_film_64x48s8", (64, 48), 8, 0, 3, tmp, scene=sc)
    paths_fixture("imagemap_paths_96x72s2_seed5", (96, 72), 2, 5, 3, 2, tmp, scene=sc)


def textured_fixtures(tmp):
    """tests/scenes/textured.pbrt: every material parameter as a texture -- two textured spectra
    per material, textured roughness / sigma / u-v roughness / index, metal's unclamped eta and k"""
    sc = os.path.join(ROOT, "tests", "scenes", "textured.pbrt")
    paths_fixture("textured_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("textured_film_64x48s8", (64, 48), 8, 0, 5, tmp, scene=sc)
    paths_fixture("textured_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc,
                  extra=("--surf", "directlighting", "--dl-strategy", "all"))
    film_fixture("textured_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc,
                 extra=("--surf", "directlighting", "--dl-strategy", "all"))


def lights_fixtures(tmp):
    """tests/scenes/lights.pbrt: spot lights (falloff band, transformed frames) and a distant light
    next to an area light; path and DirectLighting, the spectral and the RGB build"""
    sc = os.path.join(ROOT, "tests", "scenes", "lights.pbrt")
    paths_fixture("lights_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("lights_film_64x48s8", (64, 48), 8, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("lights_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("lights_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)
    if os.path.exists(HARNESSRGB):
        paths_fixture("lights_rgb_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc, bands=3)
        film_fixture("lights_rgb_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc, bands=3)


def ortho_fixtures(tmp):
    """tests/scenes/ortho.pbrt: the orthographic camera (screen window, thin lens, shutter) over a
    textured, bump-mapped floor (its ray differentials); path and DirectLighting"""
    sc = os.path.join(ROOT, "tests", "scenes", "ortho.pbrt")
    paths_fixture("ortho_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("ortho_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("ortho_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("ortho_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)


def heightfield_fixtures(tmp):
    """tests/scenes/heightfield.pbrt: heightfield shapes (terrain, area light) refined as the
    reference does; path integrator and the metadata integrator's mesh ids"""
    sc = os.path.join(ROOT, "tests", "scenes", "heightfield.pbrt")
    paths_fixture("heightfield_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("heightfield_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "metadata", "--meta-strategy", "mesh")
    paths_fixture("heightfield_meta_mesh_paths_48x36s2", (48, 36), 2, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("heightfield_meta_mesh_film_48x36s2", (48, 36), 2, 0, 5, tmp, scene=sc, extra=ex)


def cylinder_fixtures(tmp):
    """tests/scenes/cylinder.pbrt: cylinders (phimax cut, both roots, textured, reversed, an area
    light); path and DirectLighting"""
    sc = os.path.join(ROOT, "tests", "scenes", "cylinder.pbrt")
    paths_fixture("cylinder_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("cylinder_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("cylinder_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("cylinder_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)


def anisoward_fixtures(tmp):
    """tests/scenes/anisoward.pbrt: the fork's anisotropic Ward material (constant, anisotropic,
    textured parameters); path and DirectLighting, and the RGB build"""
    sc = os.path.join(ROOT, "tests", "scenes", "anisoward.pbrt")
    paths_fixture("anisoward_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("anisoward_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("anisoward_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("anisoward_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)


def mappings_fixtures(tmp):
    """tests/scenes/mappings.pbrt: the spherical / cylindrical / planar 2D texture mappings
    (texture.cpp:93-144) on image textures and bump maps; path and DirectLighting"""
    sc = os.path.join(ROOT, "tests", "scenes", "mappings.pbrt")
    paths_fixture("mappings_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("mappings_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("mappings_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("mappings_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)


def checker_fixtures(tmp):
    """tests/scenes/checker.pbrt: Checkerboard2DTexture (checkerboard.h:84-125) with its mappings and
    operands; path and DirectLighting"""
    sc = os.path.join(ROOT, "tests", "scenes", "checker.pbrt")
    paths_fixture("checker_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("checker_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("checker_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("checker_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)


def shinymetal_fixtures(tmp):
    """tests/scenes/shinymetal.pbrt: shinymetal's conductor microfacet and mirror lobes (FresnelApproxEta
    of constant Ks / Kr); path and DirectLighting (its specular recursion)"""
    sc = os.path.join(ROOT, "tests", "scenes", "shinymetal.pbrt")
    paths_fixture("shinymetal_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("shinymetal_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "directlighting", "--dl-strategy", "all")
    paths_fixture("shinymetal_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("shinymetal_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc, extra=ex)


def nurbs_fixtures(tmp):
    """tests/scenes/nurbs.pbrt: NURBS patches (P and rational Pw, interior knots, a u range) refined as
    the reference refines them; path integrator and metadata mesh ids"""
    sc = os.path.join(ROOT, "tests", "scenes", "nurbs.pbrt")
    paths_fixture("nurbs_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("nurbs_film_64x48s4", (64, 48), 4, 0, 5, tmp, scene=sc)
    ex = ("--surf", "metadata", "--meta-strategy", "mesh")
    paths_fixture("nurbs_meta_mesh_paths_48x36s2", (48, 36), 2, 0, 5, 1, tmp, scene=sc, extra=ex)
    film_fixture("nurbs_meta_mesh_film_48x36s2", (48, 36), 2, 0, 5, tmp, scene=sc, extra=ex)


def envmap_fixtures(tmp):
    """tests/scenes/envmap.pbrt: an image-based InfiniteAreaLight (a decoded PFM lat-long map: its
    radiance MIPMap and Distribution2D), path integrator and DirectLighting"""
    sc = os.path.join(ROOT, "tests", "scenes", "envmap.pbrt")
    paths_fixture("envmap_paths_64x48s4", (64, 48), 4, 0, 5, 1, tmp, scene=sc)
    film_fixture("envmap_film_64x48s8", (64, 48), 8, 0, 5, tmp, scene=sc)
    paths_fixture("envmap_dl_paths_48x36s4", (48, 36), 4, 0, 5, 1, tmp, scene=sc,
                  extra=("--surf", "directlighting", "--dl-strategy", "all"))
    film_fixture("envmap_dl_film_48x36s4", (48, 36), 4, 0, 5, tmp, scene=sc,
                 extra=("--surf", "directlighting", "--dl-strategy", "all"))


def animcam_fixtures(tmp):
    """tests/scenes/animcam.pbrt: an animated CameraToWorld (coverage.pbrt's world)"""
    sc = os.path.join(ROOT, "tests", "scenes", "animcam.pbrt")
    paths_fixture("animcam_paths_64x48s4", (64, 48), 4, 0, 6, 2, tmp, scene=sc)
    film_fixture("animcam_film_64x48s4", (64, 48), 4, 0, 6, tmp, scene=sc)


def gpupath_fixture(tmp):
    """The .dat the reference's own spectral film (SpectralImageNoCameraFilm, --refdat) writes for
    tests/scenes/coverage.pbrt rendered by the harness on the CPU (the scene's own integrator):
    tests/test_binding_gpu.py renders the same film through Renderer "gpupath" on the GPU, which
    hands its frame to that film class and lets its WriteImage write the file."""
    cov = os.path.join(ROOT, "tests", "scenes", "coverage.pbrt")
    fn = os.path.join(tmp, "gp.dat")
    subprocess.run([HARNESS, cov, "--res", "40", "32", "--spp", "4", "--seed", "0", "--surf", "scene", "--refdat", fn],
                   check=True, cwd=tmp)
    np.savez_compressed(os.path.join(OUT, "coverage_gpupath_dat_40x32s4.npz"),
                        dat=np.frombuffer(open(fn, "rb").read(), np.uint8), config=np.array([40, 32, 4, 0, -1], np.int32))
    print("coverage_gpupath_dat_40x32s4")


def main():
    if not os.path.exists(HARNESS):
        sys.exit("build the reference harness first: make -C oracle ref")
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[2] if len(sys.argv) > 2 and sys.argv[1] == "--only" else None
    if only:
        with tempfile.TemporaryDirectory() as tmp:
            if only == "keys":
                for cfg in KEY_CONFIGS:
                    if cfg[5] == 60 and not os.path.exists(HARNESS60):
                        sys.exit("make -C oracle ref60 first")
                    keys_fixture(*cfg, tmp)
            elif only == "dat":
                dat_fixture("killeroo_dat_40x32s4", (40, 32), 4, tmp)
            elif only == "merl":
                merl_fixtures(tmp)
            elif only == "dl":
                dl_fixtures(tmp)
            elif only == "meta":
                meta_fixtures(tmp)
            elif only == "spec":
                spec_fixtures(tmp)
            elif only == "rgb":
                rgb_fixtures(tmp)
            elif only == "nurbs":
                nurbs_fixtures(tmp)
            elif only == "mappings":
                mappings_fixtures(tmp)
            elif only == "checker":
                checker_fixtures(tmp)
            elif only == "shinymetal":
                shinymetal_fixtures(tmp)
            elif only == "anisoward":
                anisoward_fixtures(tmp)
            elif only == "cylinder":
                cylinder_fixtures(tmp)
            elif only == "heightfield":
                heightfield_fixtures(tmp)
            elif only == "ortho":
                ortho_fixtures(tmp)
            elif only == "lights":
                lights_fixtures(tmp)
            elif only == "rgbfeat":
                rgbfeat_fixtures(tmp)
            elif only == "b30":
                b30_fixtures(tmp)
            elif only == "imagemap":
                imagemap_fixtures(tmp)
            elif only == "animcam":
                animcam_fixtures(tmp)
            elif only == "gpupath":
                gpupath_fixture(tmp)
            elif only == "textured":
                textured_fixtures(tmp)
            elif only == "envmap":
                envmap_fixtures(tmp)
            elif only == "window":
                sel = sys.argv[3:]
                for cfg in WINDOW_CONFIGS:
                    if not sel or cfg[0] in sel:
                        window_fixture(*cfg, tmp)
        return
    with tempfile.TemporaryDirectory() as tmp:
        paths_fixture("killeroo_paths_64x64s4", (64, 64), 4, 0, 5, 5, tmp)
        paths_fixture("killeroo_paths_48x48s8_seed7_md7", (48, 48), 8, 7, 7, 3, tmp)
        film_fixture("killeroo_film_96x72s16", (96, 72), 16, 0, 5, tmp)
        paths_fixture("anim_paths_48x48s4", (48, 48), 4, 0, 5, 3, tmp, scene="anim-killeroos-moving.pbrt")
        film_fixture("anim_film_40x40s8", (40, 40), 8, 0, 5, tmp, scene="anim-killeroos-moving.pbrt")
        paths_fixture("bunny_paths_64x36s4", (64, 36), 4, 0, 5, 3, tmp, scene="bunny.pbrt")
        film_fixture("bunny_film_48x27s8", (48, 27), 8, 0, 5, tmp, scene="bunny.pbrt")
        cov = os.path.join(ROOT, "tests", "scenes", "coverage.pbrt")
        paths_fixture("coverage_paths_64x48s8", (64, 48), 8, 0, 6, 2, tmp, scene=cov)
        film_fixture("coverage_film_64x48s8", (64, 48), 8, 0, 6, tmp, scene=cov)
        if os.path.exists(HARNESS60):
            paths_fixture("metal_paths_48x48s4", (48, 48), 4, 0, 5, 2, tmp, scene="metal.pbrt", bands=60)
            film_fixture("metal_film_40x40s8", (40, 40), 8, 0, 5, tmp, scene="metal.pbrt", bands=60)
            fn = os.path.join(tmp, "spec60.bin")
            run(["-", "--spectra", fn], 60)
            raw = np.fromfile(fn, dtype=np.int32)
            n = raw[0]
            rec = raw[1:].reshape(n, 3 + 60 + 60).view(np.float32)
            np.savez_compressed(os.path.join(OUT, "fromrgb_60.npz"), rgb=rec[:, :3].copy(), refl=rec[:, 3:63].copy(),
                                illum=rec[:, 63:].copy())
        for cfg in KEY_CONFIGS:
            if cfg[5] != 60 or os.path.exists(HARNESS60):
                keys_fixture(*cfg, tmp)
        dat_fixture("killeroo_dat_40x32s4", (40, 32), 4, tmp)
        for cfg in WINDOW_CONFIGS:
            if cfg[5] != 60 or os.path.exists(HARNESS60):
                window_fixture(*cfg, tmp)
        merl_fixtures(tmp)
        imagemap_fixtures(tmp)
        animcam_fixtures(tmp)
        gpupath_fixture(tmp)
        textured_fixtures(tmp)
        envmap_fixtures(tmp)
        dl_fixtures(tmp)
        meta_fixtures(tmp)
        spec_fixtures(tmp)
        if os.path.exists(HARNESSRGB):
            rgb_fixtures(tmp)
        if os.path.exists(HARNESS30):
            b30_fixtures(tmp)
        fn = os.path.join(tmp, "mt.bin")
        run(["-", "--kat-mt", fn])
        raw = np.fromfile(fn, dtype=np.uint32).reshape(6, 65)
        np.savez_compressed(os.path.join(OUT, "mt19937_kat.npz"), seeds=raw[:, 0].copy(), out=raw[:, 1:].copy())
        fn = os.path.join(tmp, "spec.bin")
        run(["-", "--spectra", fn])
        raw = np.fromfile(fn, dtype=np.int32)
        n = raw[0]
        rec = raw[1:].reshape(n, 3 + 32 + 32).view(np.float32)
        np.savez_compressed(os.path.join(OUT, "fromrgb_32.npz"), rgb=rec[:, :3].copy(), refl=rec[:, 3:35].copy(),
                            illum=rec[:, 35:].copy())
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
