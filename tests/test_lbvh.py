"""GPU BVH build (pbrtgpu_build_bvh, csrc/lbvh.hip).  The host front end's
SAH build restates accelerators/bvh.cpp:145-351 node for node and stays the default; the GPU
linear BVH is the opt-in fast build.  Checked here:
  * CPU: the primitive bounds it starts from cover the reference BVH's root bound;
  * GPU: the tree is well formed (every primitive in exactly one leaf, every node bound
    encloses its children, depth-first layout), the build is deterministic, traversal over it
    gives the same closest-hit t as over the reference BVH for every ray (the primitive only
    differs on exact ties), and the GPU path tracer over it equals the oracle over the same
    BVH bit for bit and the reference-BVH render up to those ties."""
import os

import numpy as np
import pytest

from conftest import PACKS


def _rays(n, seed=7):
    rng = np.random.RandomState(seed)
    lo = np.array([-1000, -1000, -140], np.float32)
    hi = np.array([1000, 1000, 200], np.float32)
    o = lo + (hi - lo) * rng.rand(n, 3).astype(np.float32)
    d = rng.randn(n, 3).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d, np.zeros((n, 1), np.float32), np.full((n, 1), np.inf, np.float32)], axis=1)


def _nodes(pg, scene):
    f = scene.flat
    a = pg._arr(f.nodes, pg.ctypes.c_uint32, 8 * f.n_nodes).reshape(-1, 8)
    return a[:, :6].view(np.float32), a[:, 6], a[:, 7]


@pytest.mark.parametrize("pack", ["killeroo-simple.pack", "coverage.pack", "bunny.pack"])
def test_prim_bounds_cover_reference_root(pg, pack):
    s = pg.Scene.load(os.path.join(PACKS, pack))
    b = pg.prim_bounds(s)
    assert b.shape == (s.flat.n_prims, 6) and np.all(b[:, :3] <= b[:, 3:])
    bb, _, _ = _nodes(pg, s)
    root = bb[0]
    lo, hi = b[:, :3].min(axis=0), b[:, 3:].max(axis=0)
    assert np.all(lo <= root[:3]) and np.all(hi >= root[3:])
    ext = np.maximum(root[3:] - root[:3], 1.0)
    assert np.all(root[:3] - lo <= 1e-5 * ext) and np.all(hi - root[3:] <= 1e-5 * ext)


def test_prim_bounds_refuse_instances(pg):
    s = pg.Scene.load(os.path.join(PACKS, "anim-killeroos-moving.pack"))
    with pytest.raises(ValueError):
        pg.prim_bounds(s)


def _check_tree(pg, scene, bvh):
    n = scene.flat.n_prims
    bb, off, meta = _nodes(pg, bvh)
    assert len(bb) == 2 * n - 1
    leaf = (meta & 0xff) != 0
    assert np.all((meta[leaf] & 0xff) == 1) and leaf.sum() == n
    assert sorted(off[leaf].tolist()) == list(range(n))          # each leaf position once
    assert sorted(bvh.order.tolist()) == list(range(n))         # a permutation of the prims
    b = pg.prim_bounds(scene)
    # leaf bound = its primitive's bound; interior: children next / at offset, bounds enclose
    assert np.array_equal(bb[leaf], b[bvh.order[off[leaf]]])
    inner = np.nonzero(~leaf)[0]
    for ch in (inner + 1, off[inner].astype(np.int64)):
        assert np.all(ch > inner) and np.all(ch < len(bb))
        assert np.all(bb[ch][:, :3] >= bb[inner][:, :3]) and np.all(bb[ch][:, 3:] <= bb[inner][:, 3:])


@pytest.mark.gpu
@pytest.mark.parametrize("pack", ["killeroo-simple.pack", "coverage.pack"])
def test_gpu_bvh_well_formed_and_deterministic(pg, pack):
    s = pg.Scene.load(os.path.join(PACKS, pack))
    with pg.Device(0) as d:
        b1, b2 = d.build_bvh(s), d.build_bvh(s)
    _check_tree(pg, s, b1)
    assert np.array_equal(b1._nodes, b2._nodes) and np.array_equal(b1.order, b2.order)
    print("%s: %d prims, build %.2f ms device, %.2f ms call" % (pack, s.flat.n_prims, *b1.build_ms))


@pytest.mark.gpu
def test_gpu_bvh_small_counts(pg):
    """1, 2 and 3 primitives (the root is a leaf / one interior node)."""
    s = pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"))
    rng = np.random.RandomState(3)
    with pg.Device(0) as d:
        for n in (1, 2, 3, 17):
            lo = rng.rand(n, 3).astype(np.float32)
            b = np.ascontiguousarray(np.concatenate([lo, lo + 0.1], axis=1))
            nodes = np.zeros(2 * n - 1, dtype=np.dtype([("bmin", "<f4", 3), ("bmax", "<f4", 3), ("offset", "<u4"), ("meta", "<u4")]))
            order = np.zeros(n, np.int32)
            assert d.lib.pbrtgpu_build_bvh(d.ctx, n, b.ctypes.data, nodes.ctypes.data, order.ctypes.data, None) == 2 * n - 1
            assert sorted(order.tolist()) == list(range(n))
            assert np.allclose(nodes["bmin"][0], lo.min(axis=0)) and np.allclose(nodes["bmax"][0], (lo + 0.1).max(axis=0))
        assert d.lib.pbrtgpu_build_bvh(d.ctx, 0, b.ctypes.data, nodes.ctypes.data, order.ctypes.data, None) < 0
    del s


@pytest.mark.gpu
def test_gpu_bvh_closest_hits_match_reference_bvh(pg):
    s = pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"))
    rays = _rays(100000)
    with pg.Device(0) as d:
        bvh = d.build_bvh(s)
        d.upload(s)
        h0, o0 = d.intersect(rays)
        d.upload(bvh)
        h1, o1 = d.intersect(rays)
    hit0, hit1 = h0[:, 3].view(np.int32) >= 0, h1[:, 3].view(np.int32) >= 0
    assert np.array_equal(hit0, hit1) and np.array_equal(o0, o1)
    assert np.array_equal(h0[:, 0].view(np.int32), h1[:, 0].view(np.int32))        # t, bit for bit
    p0, p1 = h0[hit0, 3].view(np.int32), bvh.order[h1[hit1, 3].view(np.int32)]
    same = p0 == p1
    assert same.mean() >= 0.999, "same primitive %d/%d" % (same.sum(), len(same))
    # the oracle over the GPU-built BVH: the same traversal, bit for bit
    ho, oo = pg.oracle().intersect(bvh, rays)
    assert np.array_equal(h1.view(np.int32), ho.view(np.int32)) and np.array_equal(o1, oo)


@pytest.mark.gpu
def test_gpu_bvh_paths(pg):
    s = pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"), xres=48, yres=48, spp=4)
    c = s.flat.camera
    keys = np.array([(x, y, k) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
                     for k in range(s.spp)], np.int32)
    with pg.Device(0) as d:
        bvh = d.build_bvh(s)
        d.upload(s)
        L0 = d.trace_paths(keys)
        d.upload(bvh)
        L1 = d.trace_paths(keys)
    Lo = pg.oracle().trace_paths(bvh, keys)
    from conftest import assert_bit_exact
    assert_bit_exact(L1, Lo, "GPU vs oracle over the GPU BVH")
    exact_r = np.all(L1.view(np.int32) == L0.view(np.int32), axis=1)
    assert exact_r.mean() >= 0.999, "GPU BVH vs reference BVH: %d/%d" % (exact_r.sum(), len(keys))
