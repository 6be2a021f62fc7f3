"""GPU Loop subdivision (pbrtgpu_loop_subdivide, csrc/loopsubdiv.hip)
against the front end's restatement of LoopSubdiv::Refine (host/frontend.cpp LoopRefineCore,
which the reference-derived scene packs pin: the killeroos of every config are refined by it).
Positions and faces must be bit-identical; normals use cosf / sinf, whose GPU restatement may
differ from glibc in the last ulp."""
import os

import numpy as np
import pytest

from conftest import ROOT
from loop_meshes import MESHES

SCENE = os.path.join(ROOT, "tests", "scenes", "loop.pbrt")


@pytest.mark.parametrize("name", sorted(MESHES))
def test_host_refine_sizes(pg, name):
    F, P = MESHES[name]()
    for levels in (0, 1, 2):
        Po, No, vo = pg.loop_refine_host(F, P, levels)
        assert vo.shape == (len(F) << (2 * levels), 3)
        assert vo.min() >= 0 and vo.max() == len(Po) - 1
        assert np.isfinite(Po).all() and np.isfinite(No).all()


def test_loop_scene_loads_on_host(pg):
    s = pg.Scene.load(SCENE)
    assert s.flat.n_tris >= (20 + 32) * 64 + 1   # two 3-level surfaces and the light


def _cmp(a, b):
    return np.all(a.view(np.int32) == b.view(np.int32), axis=1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MESHES))
def test_gpu_loop_matches_host(pg, name):
    F, P = MESHES[name]()
    with pg.Device(0) as d:
        for levels in (0, 1, 2, 3):
            Ph, Nh, vh = pg.loop_refine_host(F, P, levels)
            Pg, Ng, vg = d.loop_subdivide(F, P, levels)
            assert np.array_equal(vg, vh), "faces, %d levels" % levels
            assert _cmp(Pg, Ph).all(), "limit positions, %d levels: %d/%d" % (levels, _cmp(Pg, Ph).sum(), len(Ph))
            en = _cmp(Ng, Nh)
            assert en.all(), "normals, %d levels: %d/%d" % (levels, en.sum(), len(en))


@pytest.mark.gpu
def test_gpu_loop_rejects_bad_meshes(pg):
    F, P = MESHES["tetrahedron"]()
    with pg.Device(0) as d:
        with pytest.raises(RuntimeError):
            d.loop_subdivide(F, np.concatenate([P, [[5, 5, 5]]]), 1)   # a vertex of no face
        with pytest.raises(RuntimeError):
            d.loop_subdivide(np.array([[0, 1, 9]], np.int32), P, 1)     # index out of range


@pytest.mark.gpu
def test_front_end_refines_on_the_gpu(pg):
    """pbrthost_set_loop_subdivider + pbrtgpu_loop_subdivide_hook: the scene's loopsubdiv
    shapes refined on the GPU give the same flattened scene as the host refinement."""
    h = pg.Scene.load(SCENE)
    with pg.Device(0) as d:
        pg.use_gpu_subdivision(d)
        try:
            g = pg.Scene.load(SCENE)
        finally:
            pg.use_gpu_subdivision(None)
    fh, fg = h.flat, g.flat
    assert fh.n_tris == fg.n_tris and fh.n_verts == fg.n_verts and fh.n_nodes == fg.n_nodes
    n = fh.n_verts
    ph, pg_ = pg._arr(fh.vert_p, pg.ctypes.c_float, 3 * n), pg._arr(fg.vert_p, pg.ctypes.c_float, 3 * n)
    assert np.array_equal(ph.view(np.int32), pg_.view(np.int32))
    nh, ng = pg._arr(fh.vert_n, pg.ctypes.c_float, 3 * n), pg._arr(fg.vert_n, pg.ctypes.c_float, 3 * n)
    assert np.array_equal(nh.view(np.int32), ng.view(np.int32))
    th, tg = pg._arr(fh.tris, pg.ctypes.c_int32, 4 * fh.n_tris), pg._arr(fg.tris, pg.ctypes.c_int32, 4 * fg.n_tris)
    assert np.array_equal(th, tg)


def _killeroo():
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "killeroo_control.npz"))
    return z["vi"], z["P"], int(z["levels"])


def test_killeroo_control_mesh_host(pg):
    F, P, levels = _killeroo()
    Ph, Nh, vh = pg.loop_refine_host(F, P, levels)
    assert len(vh) == 4 * len(F)


@pytest.mark.gpu
def test_gpu_loop_killeroo(pg):
    """The reference's killeroo control mesh at its own level count and two more: GPU = host,
    and the timing of both (printed; profiles/r02q_loop.json)."""
    import time
    F, P, levels = _killeroo()
    with pg.Device(0) as d:
        d.loop_subdivide(F, P, 1)   # warm-up (module load)
        for lv in (levels, levels + 1, levels + 2):
            t0 = time.perf_counter(); Ph, Nh, vh = pg.loop_refine_host(F, P, lv); th = time.perf_counter() - t0
            t0 = time.perf_counter(); Pg, Ng, vg = d.loop_subdivide(F, P, lv); tg = time.perf_counter() - t0
            assert np.array_equal(vg, vh) and _cmp(Pg, Ph).all()
            en = _cmp(Ng, Nh)
            print("killeroo %d levels: %d verts, %d faces; host %.1f ms, GPU %.1f ms (call); normals bit-exact %.6f"
                  % (lv, len(Ph), len(vh), 1e3 * th, 1e3 * tg, en.mean()))
            assert en.all()
