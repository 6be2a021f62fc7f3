"""The GPU's device shading code replayed on the CPU (tools/hostsan/shade_host.cpp) against the
oracle, and under the host sanitizers.

shade_host compiles csrc/wavefront.h, directlighting.h, metadata.h, device.h and scene_build.h
as host C++ (tools/hostsan/hip/hip_runtime.h stands in for the HIP header) and drives the
wavefront pass by pass as pbrtgpu.hip does.  It is test infrastructure: these tests pin the
device source itself, independently of the GPU --
  * bit-exact with the C oracle (liboracle.so, the transcendental definition the GPU uses) for
    every integrator and the packaged scenes, and at config C2's real size (golden keys);
  * no read of state a pass did not write: MSan reports none, and the radiance does not change
    with the byte the path-slot arrays are filled with (--poison);
  * no out-of-bounds access or undefined behaviour: ASan + UBSan report none.
This is how the DirectLighting non-determinism of the first 3-wave build was localised to that
build's machine code rather than its source.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PACKS, ROOT

HS = os.path.join(ROOT, "tools", "hostsan")
# the RealisticDiffractionCamera with diffraction on (an absolute path: os.path.join keeps it)
LENS_D = os.path.join(ROOT, "tests", "scenes", "lens_diffraction.pbrt")
# its light-field modes (pinhole array; microlenses with diffraction) and the schematic eye
LF_P = os.path.join(ROOT, "tests", "scenes", "lens_pinholes.pbrt")
LF_M = os.path.join(ROOT, "tests", "scenes", "lens_microlens.pbrt")
EYE = os.path.join(ROOT, "tests", "scenes", "eye.pbrt")
SCN = os.path.join(ROOT, "tests", "scenes", "")


def _build(target):
    subprocess.run(["make", "-s", "-C", HS, target], check=True, capture_output=True)
    return os.path.join(HS, target)


def _keys(scene):
    c = scene.flat.camera
    return np.array([(x, y, s) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
                     for s in range(scene.spp)], np.int32)


def _replay(exe, pack, tmp_path, keys=None, poison=None, **a):
    out = str(tmp_path / "L.f32")
    cmd = [exe, pack, "--out", out]
    for k, v in a.items():
        cmd += ["--" + k, str(v)]
    if poison is not None:
        cmd += ["--poison", str(poison)]
    if keys is not None:
        kf = str(tmp_path / "keys.i32")
        np.ascontiguousarray(keys, np.int32).tofile(kf)
        cmd += ["--keys", kf]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: MemorySanitizer", "LeakSanitizer"):
        assert bad not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stderr[-4000:]
    return np.fromfile(out, np.float32)


CASES = [
    ("coverage.pack", dict(xres=40, yres=30, spp=4, maxdepth=6, integrator="directlighting", strategy="all")),
    ("coverage.pack", dict(xres=40, yres=30, spp=4, maxdepth=5, integrator="directlighting", strategy="one")),
    ("killeroo-simple.pack", dict(xres=32, yres=24, spp=4, maxdepth=5, integrator="directlighting", strategy="all")),
    ("coverage.pack", dict(xres=40, yres=30, spp=8, maxdepth=5)),
    ("anim-killeroos-moving.pack", dict(xres=24, yres=24, spp=4, maxdepth=5)),
    ("bunny.pack", dict(xres=24, yres=16, spp=4, maxdepth=5)),
    ("metal.pack", dict(xres=24, yres=24, spp=4, maxdepth=5)),
    ("coverage.pack", dict(xres=40, yres=30, spp=2, integrator="metadata", strategy="depth")),
    ("coverage-b30.pack", dict(xres=40, yres=30, spp=4, maxdepth=6)),
    (LENS_D, dict(xres=40, yres=30, spp=4, maxdepth=5)),
    (LENS_D, dict(xres=32, yres=24, spp=2, maxdepth=5, renderer="spectral", wave_bands=8, sampling="single")),
    (LF_P, dict(xres=64, yres=48, spp=2, maxdepth=5)),
    (LF_M, dict(xres=64, yres=48, spp=4, maxdepth=5, renderer="spectral", wave_bands=4, sampling="single")),
    (EYE, dict(xres=48, yres=36, spp=2, maxdepth=5)),
    (EYE, dict(xres=48, yres=36, spp=2, maxdepth=5, renderer="spectral", wave_bands=8, sampling="single")),
    (LENS_D, dict(xres=32, yres=24, spp=2, maxdepth=5, integrator="directlighting", strategy="all")),
    ("imagemap.pack", dict(xres=48, yres=36, spp=4, maxdepth=3)),
    ("imagemap.pack", dict(xres=40, yres=30, spp=2, maxdepth=3, integrator="directlighting", strategy="all")),
    ("animcam.pack", dict(xres=40, yres=30, spp=4, maxdepth=6)),
    ("textured.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    ("textured.pack", dict(xres=32, yres=24, spp=2, maxdepth=5, integrator="directlighting", strategy="all")),
    ("envmap.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    ("envmap.pack", dict(xres=32, yres=24, spp=2, maxdepth=5, integrator="directlighting", strategy="all")),
    # DirectLighting over instances (ray slots stay per slot, terms per list row) and at 60 bands
    ("anim-killeroos-moving.pack", dict(xres=24, yres=24, spp=4, maxdepth=5, integrator="directlighting", strategy="all")),
    ("metal.pack", dict(xres=24, yres=24, spp=4, maxdepth=5, integrator="directlighting", strategy="all")),
    # the RGB build (NB = 3): image textures and normal maps, the environment map, SPD spectra
    (SCN + "imagemap.pbrt", dict(xres=40, yres=30, spp=2, maxdepth=3, bands=3)),
    (SCN + "envmap.pbrt", dict(xres=32, yres=24, spp=2, maxdepth=5, bands=3, integrator="directlighting", strategy="all")),
    (SCN + "coverage.pbrt", dict(xres=32, yres=24, spp=2, maxdepth=6, bands=3)),
    # spot and distant lights (FEAT_INF kernels) beside an area light
    ("lights.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    ("lights.pack", dict(xres=32, yres=24, spp=2, maxdepth=5, integrator="directlighting", strategy="all")),
    # shinymetal (conductor mirror lobe: FEAT_TEX kernels), with DirectLighting's specular recursion
    ("shinymetal.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    ("shinymetal.pack", dict(xres=32, yres=24, spp=2, maxdepth=5, integrator="directlighting", strategy="all")),
    # the fork's anisotropic Ward material
    ("anisoward.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    # cylinders (hit-only test shared with the sphere's, full intersection, area light)
    ("cylinder.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    ("cylinder.pack", dict(xres=32, yres=24, spp=2, maxdepth=5, integrator="directlighting", strategy="all")),
    # spherical / cylindrical / planar texture mappings (image textures, bump maps)
    ("mappings.pack", dict(xres=40, yres=30, spp=4, maxdepth=3)),
    ("mappings.pack", dict(xres=32, yres=24, spp=2, maxdepth=3, integrator="directlighting", strategy="all")),
    # Checkerboard2DTexture (closed form / point sampled, constant and image operands, mappings)
    ("checker.pack", dict(xres=40, yres=30, spp=4, maxdepth=3)),
    ("checker.pack", dict(xres=32, yres=24, spp=2, maxdepth=3, integrator="directlighting", strategy="all")),
    # NURBS patches (refined on the host into a mesh with normals)
    ("nurbs.pack", dict(xres=40, yres=30, spp=2, maxdepth=5)),
    # heightfield shapes (refined on the host; one as an area light)
    ("heightfield.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    # the orthographic camera (thin lens, ray differentials from shifted origins)
    ("ortho.pack", dict(xres=40, yres=30, spp=4, maxdepth=5)),
    # an animated CameraToWorld under the lens camera
    (SCN + "lens_animated.pbrt", dict(xres=32, yres=24, spp=2, maxdepth=5)),
]


@pytest.mark.parametrize("pack,a", CASES, ids=["dl_all_md6", "dl_one", "dl_killeroo", "path_coverage", "path_anim",
                                               "path_bunny", "path_metal60", "metadata", "path_coverage_b30",
                                               "lens_diffraction", "lens_diffraction_spectral", "lens_pinholes",
                                               "lens_microlens_spectral", "eye", "eye_spectral", "lens_diffraction_dl",
                                               "imagemap", "imagemap_dl", "animcam", "textured", "textured_dl", "envmap", "envmap_dl",
                                               "dl_anim_inst",
                                               "dl_metal60", "rgb_imagemap", "rgb_envmap_dl", "rgb_coverage", "lights", "lights_dl", "shinymetal", "shinymetal_dl", "anisoward", "cylinder", "cylinder_dl", "mappings", "mappings_dl", "checker", "checker_dl", "nurbs", "heightfield", "ortho", "lens_animated"])
def test_replay_matches_oracle(pg, tmp_path, pack, a):
    exe = _build("shade_host")
    scene = pg.Scene.load(os.path.join(PACKS, pack), **a)
    keys = _keys(scene)
    Lo = pg.oracle().trace_paths(scene, keys)
    L = _replay(exe, os.path.join(PACKS, pack), tmp_path, **a).reshape(Lo.shape)
    assert np.array_equal(L.view(np.int32), Lo.view(np.int32))


KEYS = [("killeroo_keys_c2_700x700s256", "killeroo-simple.pack"), ("bunny_keys_c3_1920x1080s1024", "bunny.pack"),
        ("metal_keys_c4_400x400s4096", "metal.pack"), ("anim_keys_c5_600x600s512", "anim-killeroos-moving.pack")]


@pytest.mark.parametrize("name,pack", KEYS, ids=["c2", "c3", "c4", "c5"])
def test_replay_config_golden_keys(pg, tmp_path, name, pack):
    """Configs C2-C5 at their real size and sample count: the reference harness's golden keys."""
    from test_oracle_golden import exact_rate
    exe = _build("shade_host")
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    w, h, spp, seed, md = [int(v) for v in g["config"]]
    assert seed == 0   # the packs' own seed
    pack = os.path.join(PACKS, pack)
    scene = pg.Scene.load(pack, xres=w, yres=h, spp=spp, maxdepth=md, seed=seed)
    Lo = pg.oracle().trace_paths(scene, g["keys"])
    L = _replay(exe, pack, tmp_path, keys=g["keys"], xres=w, yres=h, spp=spp, maxdepth=md).reshape(Lo.shape)
    assert np.array_equal(L.view(np.int32), Lo.view(np.int32))
    assert np.all(L.view(np.int32) == g["L"].view(np.int32), axis=1).mean() >= exact_rate(name)


def test_kd_radius_closed_form():
    """wavefront.h kd_radius_of (no loop) equals the reference retry loop's final radius
    (IrregIsotropicBRDF::f, measured.cpp) over every non-negative float"""
    exe = _build("shade_host")
    r = subprocess.run([exe, "--kd-radius-check"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr


def test_scale_inverse_fast_path():
    """device.h m4_inverse_scale (a diagonal AnimatedTransform scale factor inverted directly)
    gives the general Gauss-Jordan m4_inverse's bits (transform.cpp:68-130) on 2 M matrices"""
    exe = _build("shade_host")
    r = subprocess.run([exe, "--m4inv-check"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "mismatches 0 " in r.stdout, r.stdout + r.stderr


def test_device_rng_matches_oracle(pg, tmp_path):
    """device.h's MT19937 (5-word window, then the full state rebuilt at output 227 and twisted
    every 624) against the oracle's, over 4 generations."""
    exe = _build("shade_host")
    out = str(tmp_path / "mt.u32")
    for seed in (0, 1, 5489, 123456789, 0xdeadbeef):
        subprocess.run([exe, str(seed), "--mt-kat", "2600", "--out", out], check=True, capture_output=True)
        assert np.array_equal(np.fromfile(out, np.uint32), pg.oracle().mt_first(seed, 2600))


@pytest.mark.parametrize("md,strategy", [(16, "all"), (20, "one")])
def test_replay_deep_directlighting(pg, tmp_path, md, strategy):
    """DirectLighting recursion deep enough that paths draw past the RNG's first 227 outputs."""
    exe = _build("shade_host")
    a = dict(xres=40, yres=30, spp=4, maxdepth=md, integrator="directlighting", strategy=strategy)
    pack = os.path.join(PACKS, "coverage.pack")
    scene = pg.Scene.load(pack, **a)
    Lo = pg.oracle().trace_paths(scene, _keys(scene))
    L = _replay(exe, pack, tmp_path, **a).reshape(Lo.shape)
    assert np.array_equal(L.view(np.int32), Lo.view(np.int32))


def test_replay_independent_of_unwritten_state(pg, tmp_path):
    """Path-slot arrays filled with 0x00, 0xff or 0x7f (NaN patterns) before the run: the same bits."""
    exe = _build("shade_host")
    pack, a = CASES[0]
    runs = [_replay(exe, os.path.join(PACKS, pack), tmp_path, poison=p, **a) for p in (0x00, 0xff, 0x7f)]
    pack2, a2 = CASES[3]
    runs2 = [_replay(exe, os.path.join(PACKS, pack2), tmp_path, poison=p, **a2) for p in (0x00, 0xff, 0x7f)]
    for r in runs[1:]:
        assert np.array_equal(r.view(np.int32), runs[0].view(np.int32))
    for r in runs2[1:]:
        assert np.array_equal(r.view(np.int32), runs2[0].view(np.int32))


@pytest.mark.parametrize("variant", ["shade_host_asan", "shade_host_msan"])
def test_replay_under_sanitizers(pg, tmp_path, variant):
    """Every case above (DirectLighting's specular recursion and light-sample batches, the path
    integrator on every packaged scene and coverage.pbrt's features, metadata) under ASan + UBSan
    and under MSan: no report, oracle bits."""
    exe = _build(variant)
    for pack, a in CASES:
        scene = pg.Scene.load(os.path.join(PACKS, pack), **a)
        Lo = pg.oracle().trace_paths(scene, _keys(scene))
        L = _replay(exe, os.path.join(PACKS, pack), tmp_path, **a).reshape(Lo.shape)
        assert np.array_equal(L.view(np.int32), Lo.view(np.int32))


def test_scene_check_refuses_leaf_kinds_the_device_cannot_evaluate(pg, tmp_path):
    """scene_check (scene_build.h) admits as leaves of a combining texture (SCALE, MIX, CHECKER,
    DOTS) only the kinds the device evaluates there: a spectral SCALE over a noise node (whose
    `levels` is an octave count and whose width / height are 0) would reach tex_image<3> through
    spec_leaf -> leaf_rgb and index texels[] modulo 0.  The front end never builds that graph; a
    pack is untrusted input, so the check refuses it before any upload (the host replay runs the
    same scene_check the GPU upload does)."""
    import ctypes
    exe = _build("shade_host")
    s = pg.Scene.load(os.path.join(PACKS, "textured.pack"), xres=8, yres=6, spp=1)
    f = s.flat
    rec = np.frombuffer((ctypes.c_char * (f.n_textures * 148)).from_address(f.textures), dtype=np.int32).reshape(-1, 37)
    scale = [i for i in range(f.n_textures) if rec[i, 0] == 2 and rec[i, 1] == 1]   # spectral SCALE nodes
    assert scale
    t1, t2 = rec[scale[0], 2], rec[scale[0], 3]
    leaf = t1 if rec[t1, 0] != 0 else t2          # its image leaf (the other one is the CONST)
    ok = str(tmp_path / "ok.pack")
    s.save_pack(ok)
    _replay(exe, ok, tmp_path)                     # as built: admitted and rendered
    rec[leaf, 0] = 7                               # PBRTGPU_TEX_FBM, spectral: SCALE(FBM, CONST)
    rec[leaf, 11] = 8                              # a valid octave count: only the leaf kind is wrong
    bad = str(tmp_path / "bad.pack")
    s.save_pack(bad)
    r = subprocess.run([exe, bad, "--out", str(tmp_path / "L.f32")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "scene:" in r.stderr and "texture" in r.stderr, r.stderr[-2000:]
