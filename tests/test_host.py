"""Host front end (libpbrthost.so): scene packs, overrides, the .dat writer, and -- where
the reference's scene files exist -- parsing the unchanged pbrt scene into the same
flattened scene the committed pack holds."""
import ctypes
import os

import numpy as np
import pytest

from conftest import PACKS, REF_SCENES

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
    true by default); the eye IOR curves and pinhole arrays are refused; the .dat header's line 2
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
    src = open(os.path.join(here, "lens.pbrt")).read()
    for bad, msg in [('"bool diffractionEnabled" "false" "bool IORforEyeEnabled" "true"', "IORforEye"),
                     ('"bool diffractionEnabled" "false" "float num_pinholes_w" [4] "float num_pinholes_h" [4]',
                      "pinhole")]:
        body = src.replace('"bool diffractionEnabled" "false"', bad)
        p = os.path.join(here, "_lens_bad.pbrt")   # next to the lens file it names
        try:
            open(p, "w").write(body)
            with pytest.raises(RuntimeError, match=msg):
                pg.Scene.load(p)
        finally:
            os.remove(p)
    film = np.zeros((s.height, s.width, s.bands), np.float32)
    dat = str(tmp_path / "lens.dat")
    s.write_dat(dat, film)
    line2 = open(dat, "rb").read().split(b"\n")[1].decode()
    a = np.float32(64) / np.float32(48)
    w = np.float32(43.27) / np.sqrt(np.float32(1) + np.float32(1) / (a * a))
    fov = np.float32(2 * float(np.arctan(np.float32(w / np.float32(100.0)))) / 3.1415926539 * 180)
    assert line2 == "%g %g %g" % (50.0, f.lens.fstop, fov)


def test_rgb_build_front_end(pg):
    """bands=3 is the reference's RGB build: 'color' parameters stay RGB triples (no basis, no
    clamp), y() uses RGBSpectrum's YWeight with yint 1; what converts spectra on the device
    (image textures, the environment light) or needs sampled spectra is refused."""
    s = pg.Scene.load(os.path.join(PACKS, "killeroo-simple-rgb.pack"))
    assert s.bands == 3 and s.flat.y_int == 1.0
    y = np.ctypeslib.as_array(ctypes.cast(s.flat.band_Y, ctypes.POINTER(ctypes.c_float)), (3,))
    assert y.tolist() == [np.float32(0.212671), np.float32(0.715160), np.float32(0.072169)]
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
    with pytest.raises(RuntimeError, match="RGB build"):
        pg.Scene.load(os.path.join(here, "coverage.pbrt"), bands=3)
    assert s.flat.n_lights == 1
