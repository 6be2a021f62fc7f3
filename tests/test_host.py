"""Host front end (libpbrthost.so): scene packs, overrides, the .dat writer, and -- where
the reference's scene files exist -- parsing the unchanged pbrt scene into the same
flattened scene the committed pack holds."""
import ctypes
import os

import numpy as np
import pytest

from conftest import PACKS, REF_SCENES, ROOT

PACK = os.path.join(PACKS, "killeroo-simple.pack")


def _arr(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype)
    buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype).copy()


def flat_arrays(scene):
    f = scene.flat
    return {
        "nodes": _arr(f.nodes, f.n_nodes * 8, np.uint32),
        "prims": _arr(f.prims, f.n_prims * 4, np.int32),
        "tris": _arr(f.tris, f.n_tris * 4, np.int32),
        "vert_p": _arr(f.vert_p, f.n_verts * 3, np.uint32),
        "vert_n": _arr(f.vert_n, f.n_verts * 3, np.uint32),
        "materials": _arr(f.materials, f.n_materials * 16, np.uint32),
        "lights": _arr(f.lights, f.n_lights * 44, np.uint32),
        "spectra": _arr(f.spectra, f.n_spectra_floats, np.uint32),
        "camera": np.frombuffer(bytes(f.camera), np.uint32).copy(),
    }


def test_pack_info(pg):
    s = pg.Scene.load(PACK)
    info = s.info()
    assert (info["bands"], info["spp"], info["maxdepth"]) == (32, 256, 5)
    assert (info["width"], info["height"]) == (700, 700)
    assert info["nodes"] == 131363 and info["prims"] == 66533 and info["tris"] == 66532
    assert info["quadrics"] == 1 and info["lights"] == 1 and info["bvh_depth"] == 23


def test_pack_roundtrip(pg, tmp_path):
    s = pg.Scene.load(PACK, xres=64, yres=48, spp=8, seed=3)
    out = str(tmp_path / "rt.pack")
    s.save_pack(out)
    t = pg.Scene.load(out)
    a, b = flat_arrays(s), flat_arrays(t)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert (t.width, t.height, t.spp, t.flat.seed) == (64, 48, 8, 3)


def test_overrides(pg):
    s = pg.Scene.load(PACK, xres=100, yres=50, spp=5, maxdepth=3, seed=9)
    assert (s.width, s.height) == (100, 50)
    assert s.spp == 8                       # LDSampler rounds up to a power of two
    assert s.flat.max_depth == 3 and s.flat.seed == 9
    c = s.flat.camera
    assert (c.sx_start, c.sx_end, c.sy_start, c.sy_end) == (0, 101, 0, 51)   # box filter 0.5 border
    with pytest.raises(RuntimeError):
        pg.Scene.load(PACK, bands=60)        # a pack holds one band count


def test_bad_inputs(pg, tmp_path):
    with pytest.raises(RuntimeError):
        pg.Scene.load(str(tmp_path / "missing.pbrt"))
    bad = tmp_path / "bad.pack"
    bad.write_bytes(b"not a pack")
    with pytest.raises(RuntimeError):
        pg.Scene.load(str(bad))


def test_write_dat_layout(pg, tmp_path):
    s = pg.Scene.load(PACK, xres=6, yres=4, spp=1)
    film = np.arange(4 * 6 * 32, dtype=np.float32).reshape(4, 6, 32) - 100.0
    fn = str(tmp_path / "o.dat")
    s.write_dat(fn, film)
    raw = open(fn, "rb").read()
    l1 = raw.index(b"\n")
    l2 = raw.index(b"\n", l1 + 1)
    assert raw[:l1] == b"6 4 32"
    data = np.frombuffer(raw[l2 + 1:], dtype=np.float64)
    assert data.size == 6 * 4 * 32
    # SpectralImageFilm::WriteImage (spectralImage.cpp:267-378): the clamp to >= 0 walks a
    # running offset (x-major) while the copy is indexed y * W + x, so an entry is clamped
    # only if it was copied before the walk reached it; planes are band-major, x * H + y.
    W, H, N = 6, 4, 32
    finalC = np.zeros((W * H, N), np.float32)
    off = 0
    for x in range(W):
        for y in range(H):
            finalC[y * W + x] = film[y, x]
            finalC[off] = np.maximum(finalC[off], 0)
            off += 1
    expect = np.zeros((N, W * H))
    for x in range(W):
        for y in range(H):
            expect[:, x * H + y] = finalC[y * W + x]
    assert np.array_equal(data.reshape(N, W * H), expect)
    # line 2: focal length, f-stop, field of view of a non-RealisticDiffraction camera
    # (0, 0, 2 atan(0 / 0) ...), as the film's ofstream prints them
    assert raw[l1 + 1:l2] == b"0 0 -nan"


def test_write_dat_vs_reference_film(pg, tmp_path):
    """The .dat of the reference's own spectral film (SpectralImageNoCameraFilm, compiled from
    film/spectralImageNoCamera.cpp into the harness; same AddSample sums and WriteImage payload
    as SpectralImageFilm, spectralImage.cpp:77-152, 267-378, but no lens line) against
    pbrthost_write_dat of the harness's restatement film of the same render
    (tests/golden/killeroo_dat_40x32s4.npz, tools/make_golden.py --only dat)."""
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "killeroo_dat_40x32s4.npz"))
    film, ref = g["film"], g["dat"].tobytes()
    H, W, N = film.shape
    s = pg.Scene.load(PACK, xres=W, yres=H, spp=1)
    fn = str(tmp_path / "k.dat")
    s.write_dat(fn, film)
    mine = open(fn, "rb").read()
    r1 = ref.index(b"\n") + 1
    m1 = mine.index(b"\n") + 1
    m2 = mine.index(b"\n", m1) + 1
    assert ref[:r1] == mine[:m1] == b"%d %d %d\n" % (W, H, N)
    assert mine[m1:m2] == b"0 0 -nan\n"
    assert len(ref) - r1 == W * H * N * 8
    assert ref[r1:] == mine[m2:]          # payload bit for bit (float64 planes)


@pytest.mark.reference
def test_frontend_parses_reference_scene_to_pack(pg):
    s = pg.Scene.load(os.path.join(REF_SCENES, "killeroo-simple.pbrt"), xres=700, yres=700, spp=256)
    p = pg.Scene.load(PACK)
    a, b = flat_arrays(s), flat_arrays(p)
    for k in a:
        assert np.array_equal(a[k], b[k]), k


def test_pack_keeps_merl_tables(pg, merl_dir, tmp_path):
    """Scene packs (version 6) carry the RegularHalfangle tables; the missing-file material
    keeps aux = -1 (no BxDF)."""
    import ctypes
    s = pg.Scene.load(os.path.join(merl_dir, "merl.pbrt"), xres=16, yres=12, spp=1)
    fn = str(tmp_path / "m.pack")
    s.save_pack(fn)
    p = pg.Scene.load(fn)
    n = s.flat.n_merl_floats
    assert n == p.flat.n_merl_floats == 3 * 90 * 90 * 180
    a = np.ctypeslib.as_array(ctypes.cast(s.flat.merl, ctypes.POINTER(ctypes.c_float)), (n,))
    b = np.ctypeslib.as_array(ctypes.cast(p.flat.merl, ctypes.POINTER(ctypes.c_float)), (n,))
    assert np.array_equal(a, b) and a.min() == 0.0 and a.max() > 0.5
    mats = ctypes.cast(s.flat.materials, ctypes.POINTER(ctypes.c_int32 * 24))
    kinds = [(mats[i][0], mats[i][5]) for i in range(s.flat.n_materials)]   # (type, aux)
    assert (7, 0) in kinds and (7, -1) in kinds


def test_metadata_ids_and_text_files(pg, tmp_path):
    """pbrtWorldEnd's metadata files (api.cpp:1228-1282) list the ids the hits report: the
    quadrics' and the animated shape's primitive ids (the mesh file, scene order) and the named
    materials' ids (the materials file, by name) appear in the per-prim hit ids."""
    scn = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes", "metadata.pbrt")
    s = pg.Scene.load(scn, integrator="metadata", strategy="mesh")
    meta = s.prim_meta()
    assert meta.shape == (s.flat.n_prims, 2) and meta.min() >= 1
    # the scene file says "material": that is the strategy the text file follows
    assert s.write_metadata(str(tmp_path / "img.exr"))
    mats = [l.split() for l in open(tmp_path / "img_materials.txt").read().splitlines()]
    assert [m[1] for m in mats] == ["floor", "shiny"]
    assert {int(m[0]) for m in mats} <= set(meta[:, 1].tolist())
    # per-shape materials get fresh ids (GraphicsState::CreateMaterial), so 5 distinct ids
    assert len(set(meta[:, 1].tolist())) == 5
    pack = str(tmp_path / "m.pack")
    s.save_pack(pack)
    p = pg.Scene.load(pack)
    assert np.array_equal(p.prim_meta(), meta)
    assert p.write_metadata(str(tmp_path / "again.dat"))
    assert open(tmp_path / "again_materials.txt").read() == open(tmp_path / "img_materials.txt").read()
    # the mesh list: 5 top-level primitives in scene order; quadric / animated ids are hit ids
    d = pg.Scene.load(scn, integrator="metadata")
    d2 = str(tmp_path / "mesh.pbrt")
    open(d2, "w").write(open(scn).read().replace('"string strategy" "material"', '"string strategy" "mesh"'))
    m = pg.Scene.load(d2)
    assert m.flat.integrator == pg.INTEGRATORS["metadata"] and m.flat.meta_strategy == pg.META_STRATEGIES["mesh"]
    assert m.write_metadata(str(tmp_path / "x.exr"))
    rows = [l.split() for l in open(tmp_path / "x_mesh.txt").read().splitlines()]
    assert [r[1] for r in rows] == ["trianglemesh", "sphere", "loopsubdiv", "disk", "trianglemesh"]
    ids = set(m.prim_meta()[:, 0].tolist())
    assert int(rows[1][0]) in ids and int(rows[3][0]) in ids and int(rows[4][0]) in ids
    assert int(rows[0][0]) not in ids          # a refined mesh reports its triangles' ids
    assert d.flat.meta_strategy == pg.META_STRATEGIES["material"]


def test_spectral_renderer_directive(pg, tmp_path):
    """Renderer "spectralrenderer" (api.cpp:1377-1403): nWaveBands (default 32) and
    samplingMethod (singleDirection default, samplerDirection; others refused) reach the flat
    scene; the pack keeps them; the overrides replace them; other renderers render as sampler."""
    here = os.path.dirname(os.path.abspath(__file__))
    src = open(os.path.join(here, "scenes", "metadata.pbrt")).read()
    assert "Renderer" not in src

    def scene_with(line):
        p = tmp_path / ("r%d.pbrt" % abs(hash(line)))
        p.write_text(src.replace("WorldBegin", line + "\nWorldBegin", 1))
        return str(p)
    s = pg.Scene.load(scene_with('Renderer "spectralrenderer"'))
    assert (s.flat.renderer, s.flat.wave_bands, s.flat.spectral_sampling) == (1, 32, 0)
    assert s.paths_per_sample() == 32
    s = pg.Scene.load(scene_with('Renderer "spectralrenderer" "integer nWaveBands" [5] '
                                 '"string samplingMethod" "samplerDirection"'))
    assert (s.flat.renderer, s.flat.wave_bands, s.flat.spectral_sampling) == (1, 5, 1)
    assert s.paths_per_sample() == 1
    out = str(tmp_path / "spec.pack")
    s.save_pack(out)
    t = pg.Scene.load(out)
    assert (t.flat.renderer, t.flat.wave_bands, t.flat.spectral_sampling) == (1, 5, 1)
    t = pg.Scene.load(out, renderer="spectral", wave_bands=9, sampling="single")
    assert (t.flat.renderer, t.flat.wave_bands, t.flat.spectral_sampling) == (1, 9, 0)
    assert pg.Scene.load(out, renderer="sampler").flat.renderer == 0
    with pytest.raises(RuntimeError, match="spectral sampling"):
        pg.Scene.load(scene_with('Renderer "spectralrenderer" "string samplingMethod" "diagonal"'))
    assert pg.Scene.load(scene_with('Renderer "metropolis"')).flat.renderer == 0
    assert pg.Scene.load(PACK).flat.renderer == 0    # packs before v8: the SamplerRenderer


def test_realistic_diffraction_camera(pg, tmp_path):
    """Camera "realisticDiffraction" (realisticDiffraction.cpp:32-193): the lens file's focal
    length and elements (an aperture stop takes aperture_diameter), the camera parameters and
    its -1 shutter defaults reach the flat scene and the pack (diffractionEnabled: false here,
    true by default; no pinhole array or eye curves); the .dat header's line 2
    carries focal length, f-stop and field of view (spectralImage.cpp:356-360)."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    s = pg.Scene.load(os.path.join(here, "lens.pbrt"))
    f = s.flat
    assert f.camera_type == 1 and f.lens.n_elements == 11 and f.lens.chromatic == 1
    assert (f.lens.focal_length, f.lens.film_distance) == (50.0, np.float32(36.77))
    assert f.lens.fstop == np.float32(np.float32(50.0) / np.float32(12.0))
    el = np.ctypeslib.as_array(ctypes.cast(f.lens.elements, ctypes.POINTER(ctypes.c_float)), (11, 4))
    assert el[5].tolist() == [0.0, 4.5, 0.0, 12.0] and el[0, 0] == np.float32(29.475)
    assert (f.camera.shutter_open, f.camera.shutter_close) == (-1.0, -1.0)
    assert tuple(f.lens.pinhole_exit) == (-1.0, -1.0, -1.0)
    out = str(tmp_path / "lens.pack")
    s.save_pack(out)
    t = pg.Scene.load(out)
    el2 = np.ctypeslib.as_array(ctypes.cast(t.flat.lens.elements, ctypes.POINTER(ctypes.c_float)), (11, 4))
    assert t.flat.camera_type == 1 and np.array_equal(el, el2) and t.flat.lens.fstop == f.lens.fstop
    assert f.lens.diffraction == 0 and t.flat.lens.diffraction == 0
    assert pg.Scene.load(os.path.join(here, "lens_diffraction.pbrt")).flat.lens.diffraction == 1
    assert f.lens.num_pinholes_w == -1 and not f.lens.pinholes and not f.lens.ior_eye and not f.lens.eye_ior
    film = np.zeros((s.height, s.width, s.bands), np.float32)
    dat = str(tmp_path / "lens.dat")
    s.write_dat(dat, film)
    line2 = open(dat, "rb").read().split(b"\n")[1].decode()
    a = np.float32(64) / np.float32(48)
    w = np.float32(43.27) / np.sqrt(np.float32(1) + np.float32(1) / (a * a))
    fov = np.float32(2 * float(np.arctan(np.float32(w / np.float32(100.0)))) / 3.1415926539 * 180)
    assert line2 == "%g %g %g" % (50.0, f.lens.fstop, fov)


def test_animated_lens_camera(pg):
    """An animated CameraToWorld under the RealisticDiffractionCamera (tests/scenes/
    lens_animated.pbrt): the flat scene carries the camera's AnimatedTransform and its shutter;
    the oracle's rays take the transform at each ray's time (realisticDiffraction.cpp:1157-1158),
    so the radiance differs from the same camera held at its start transform.  PARITY UNPINNED vs
    the reference (the camera's TU needs GSL); the GPU = oracle in tests/test_gpu_parity.py."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    s = pg.Scene.load(os.path.join(here, "lens_animated.pbrt"), xres=24, yres=18, spp=2, maxdepth=4)
    f = s.flat
    assert f.camera_type == 1 and f.camera_motion
    assert (f.camera.shutter_open, f.camera.shutter_close) == (np.float32(0.1), np.float32(0.9))
    keys = np.array([(x, y, k) for y in range(0, 18, 3) for x in range(0, 24, 3) for k in range(2)], np.int32)
    o = pg.oracle()
    La = o.trace_paths(s, keys)
    s.flat.camera_motion = None   # the start transform's matrix is cam2world_m
    Ls = o.trace_paths(s, keys)
    assert np.any(La != 0) and not np.array_equal(La, Ls)


def _pinhole_array(W, H, xres, yres, film_diag, film_dist, last_ap):
    """RealisticDiffractionCamera's pinholeArray (realisticDiffraction.cpp:248-304) restated in
    numpy float32 / double arithmetic"""
    f = np.float32
    a = f(xres) / f(yres)
    width = f(film_diag) / np.sqrt(f(1) + f(1) / (a * a))
    pitch = width / f(W)
    dist = pitch * f(film_dist) / (f(last_ap) + pitch)
    pos = -f(film_dist) + dist
    out = np.zeros((W, H, 3), np.float32)
    for i in range(W):
        for j in range(H):
            cx = f(-((i - W / 2.0 + .5) * float(pitch)))
            cy = f((j - H / 2.0 + .5) * float(pitch))
            v = [f(0) - cx, f(0) - cy, f(0) + f(film_dist)]
            inv = f(1) / np.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
            d = [c * inv for c in v]
            t = pos / d[2]
            out[i, j] = (t * d[0], t * d[1], pos)
    return out


def test_light_field_and_eye_front_end(pg, tmp_path):
    """realisticDiffraction's light-field and eye parameters: "num_pinholes_w/h" (ints of floats)
    give the pinhole array, computed at the film resolution the scene is loaded with (the
    constructor's similar triangles, realisticDiffraction.cpp:248-304); "microlens_enabled";
    "IORforEyeEnabled" the four ocular IOR spectra (FromSampled band averages); packs keep them."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    for xres, yres in ((64, 48), (40, 30)):
        s = pg.Scene.load(os.path.join(here, "lens_pinholes.pbrt"), xres=xres, yres=yres)
        L = s.flat.lens
        assert (L.num_pinholes_w, L.num_pinholes_h, L.microlens, L.ior_eye) == (8, 6, 0, 0)
        ph = np.ctypeslib.as_array(ctypes.cast(L.pinholes, ctypes.POINTER(ctypes.c_float)), (8, 6, 3))
        ref = _pinhole_array(8, 6, xres, yres, 43.27, 36.77, 20.0)
        assert np.array_equal(ph.view(np.int32), ref.view(np.int32))
        assert (ph[:4, :, 0] > 0).all() and (ph[4:, :, 0] < 0).all()   # i = 0: the +x film side
    m = pg.Scene.load(os.path.join(here, "lens_microlens.pbrt"))
    assert m.flat.lens.microlens == 1 and m.flat.lens.diffraction == 1
    out = str(tmp_path / "mic.pack")
    m.save_pack(out)
    m2 = pg.Scene.load(out, xres=40, yres=30)
    assert m2.flat.lens.microlens == 1 and m2.flat.lens.num_pinholes_w == 8
    ph2 = np.ctypeslib.as_array(ctypes.cast(m2.flat.lens.pinholes, ctypes.POINTER(ctypes.c_float)), (8, 6, 3))
    assert np.array_equal(ph2, _pinhole_array(8, 6, 40, 30, 43.27, 36.77, 20.0))
    for bands in (32, 60, 30):
        e = pg.Scene.load(os.path.join(here, "eye.pbrt"), bands=bands)
        assert e.flat.lens.ior_eye == 1 and e.flat.lens.n_elements == 5
        ior = np.ctypeslib.as_array(ctypes.cast(e.flat.lens.eye_ior, ctypes.POINTER(ctypes.c_float)), (4, bands))
        # cornea, aqueous, lens, vitreous: normal dispersion (n falls with the wavelength)
        assert (np.diff(ior, axis=1) <= 1e-6).all() and (ior[:, 0] > ior[:, -1]).all()
        assert 1.37 < ior[0, bands // 2] < 1.38 and 1.41 < ior[2, bands // 2] < 1.43
        out = str(tmp_path / ("eye%d.pack" % bands))
        e.save_pack(out)
        e2 = pg.Scene.load(out)
        ior2 = np.ctypeslib.as_array(ctypes.cast(e2.flat.lens.eye_ior, ctypes.POINTER(ctypes.c_float)), (4, bands))
        assert np.array_equal(ior, ior2)
    with pytest.raises(RuntimeError, match="IORforEye|RGB build"):   # the IOR curves are SampledSpectra
        pg.Scene.load(os.path.join(here, "eye.pbrt"), bands=3)


@pytest.mark.reference
def test_eye_ior_tables_from_reference_curves(pg):
    """host/eye_ior_tables.inc (tools/gen_eye_ior.cpp) against an independent numpy float32
    restatement of Spectrum::FromSampled (AverageSpectrumSamples, spectrum.cpp:50-83) over the
    curves of the reference's realisticDiffraction.h"""
    import re
    src = open("/root/reference/src/cameras/realisticDiffraction.h").read()

    def arr(name):
        body = re.search(r"const float %s\[\d+\]\s*=\s*\{([^}]*)\}" % name, src).group(1)
        return np.array([np.float32(float(t)) for t in body.replace("\n", " ").split(",") if t.strip()], np.float32)

    f = np.float32
    lam = arr("eyeWaveSamples")
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    for bands, l0, l1 in ((32, 395, 715), (30, 400, 700)):
        e = pg.Scene.load(os.path.join(here, "eye.pbrt"), bands=bands)
        ior = np.ctypeslib.as_array(ctypes.cast(e.flat.lens.eye_ior, ctypes.POINTER(ctypes.c_float)), (4, bands))
        for k, name in enumerate(["corneaIORraw", "aqueousIORraw", "lensIORraw", "vitreousIORraw"]):
            v = arr(name)
            for i in range(bands):
                w0 = (f(1) - f(i) / f(bands)) * f(l0) + (f(i) / f(bands)) * f(l1)
                w1 = (f(1) - f(i + 1) / f(bands)) * f(l0) + (f(i + 1) / f(bands)) * f(l1)
                j = 0
                while w0 > lam[j + 1]:
                    j += 1
                acc = f(0)
                while j + 1 < len(lam) and w1 >= lam[j]:
                    a, b = max(w0, lam[j]), min(w1, lam[j + 1])

                    def interp(w):
                        t = (w - lam[j]) / (lam[j + 1] - lam[j])
                        return (f(1) - t) * v[j] + t * v[j + 1]
                    acc = acc + (f(0.5) * (interp(a) + interp(b))) * (b - a)
                    j += 1
                assert ior[k, i] == acc / (w1 - w0), (name, bands, i)


def test_rgb_build_front_end(pg):
    """bands=3 is the reference's RGB build: 'color' parameters stay RGB triples (no basis, no
    clamp), y() uses RGBSpectrum's YWeight with yint 1; sampled spectra (SPD files, the copper
    default, blackbody) go through RGBSpectrum::FromSampled, so the coverage scene loads with its
    image textures, environment light and metals (pinned by the *_rgb_* goldens)."""
    s = pg.Scene.load(os.path.join(PACKS, "killeroo-simple-rgb.pack"))
    assert s.bands == 3 and s.flat.y_int == 1.0
    y = np.ctypeslib.as_array(ctypes.cast(s.flat.band_Y, ctypes.POINTER(ctypes.c_float)), (3,))
    assert y.tolist() == [np.float32(0.212671), np.float32(0.715160), np.float32(0.072169)]
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    c = pg.Scene.load(os.path.join(here, "coverage.pbrt"), bands=3)
    assert c.bands == 3 and c.flat.n_textures > 0 and c.flat.n_lights >= 3
    assert s.flat.n_lights == 1


def test_gpupath_dat_fixture_vs_oracle(pg, tmp_path):
    """tests/golden/coverage_gpupath_dat_40x32s4.npz -- the .dat the reference's own spectral film
    wrote for tests/scenes/coverage.pbrt (the scene's path integrator, 40x32, 4 spp) -- against
    pbrthost_write_dat of the oracle's film of the same render: payload bit for bit.  This pins the
    fixture that tests/test_binding_gpu.py holds Renderer "gpupath" to on the GPU."""
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "coverage_gpupath_dat_40x32s4.npz"))
    ref = g["dat"].tobytes()
    W, H, spp = [int(v) for v in g["config"][:3]]
    s = pg.Scene.load(os.path.join(ROOT, "scenes", "coverage.pack"), xres=W, yres=H, spp=spp, seed=0)
    film, _ = pg.oracle(libm_float=True).render(s)
    fn = str(tmp_path / "c.dat")
    s.write_dat(fn, film)
    mine = open(fn, "rb").read()
    r1 = ref.index(b"\n") + 1
    m1 = mine.index(b"\n") + 1
    m2 = mine.index(b"\n", m1) + 1
    assert ref[:r1] == mine[:m1] == b"%d %d %d\n" % (W, H, s.bands)
    assert ref[r1:] == mine[m2:]


def test_pack_v15_layouts(pg):
    """Pack v16 writes the texture record's size ahead of the texture array.  pbrtgpu_texture grew
    within v15 (amount, aamode, mapping + map[16]), so a v15 pack's texture records have an
    unknown layout: a v15 pack holding textures is refused with a re-pack message, a v15 pack
    without textures loads to the same flattened scene as its v16 re-pack (fixtures: the round-5
    v15 packs of checker.pbrt and lights.pbrt, written by this front end)."""
    from conftest import GOLDEN
    with pytest.raises(RuntimeError, match="re-pack"):
        pg.Scene.load(os.path.join(GOLDEN, "pack_v15_checker.pack"))
    old = pg.Scene.load(os.path.join(GOLDEN, "pack_v15_lights.pack"))
    new = pg.Scene.load(os.path.join(PACKS, "lights.pack"))
    a, b = flat_arrays(old), flat_arrays(new)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert new.flat.n_textures == old.flat.n_textures == 0
    chk = pg.Scene.load(os.path.join(PACKS, "checker.pack"))
    assert chk.flat.n_textures > 0
