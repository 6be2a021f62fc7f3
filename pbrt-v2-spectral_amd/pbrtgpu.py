"""pbrtgpu.py -- Python plumbing over the C ABIs of libpbrthost.so / libpbrtgpu.so.

Mirrors the reference's render entry point (Renderer::Render, core/renderer.h:35-46 as
driven by pbrtWorldEnd, core/api.cpp:1287-1292) for tests and bench.py:

    scene = Scene.load("killeroo-simple.pbrt", xres=700, yres=700, spp=256)
    with Device(0) as dev:
        dev.upload(scene)
        film = dev.render()            # float32 [H][W][bands], raw sums (no normalisation)
    scene.write_dat("out.dat", film)   # SpectralImageFilm::WriteImage layout

The product path is libpbrtgpu.so: if it cannot be loaded, Device() raises -- there is no
CPU fallback.  The CPU oracle (oracle/liboracle.so) is test infrastructure and is only
loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg via oracle().
"""
import ctypes
import os
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIBDIR = os.path.join(HERE, "lib")

MAX_BANDS = 64
SHAPE_TRIANGLE, SHAPE_SPHERE, SHAPE_DISK, SHAPE_CYLINDER = 0, 1, 2, 4


class BVHNode(ctypes.Structure):
    _fields_ = [("bmin", ctypes.c_float * 3), ("bmax", ctypes.c_float * 3),
                ("offset", ctypes.c_uint32), ("meta", ctypes.c_uint32)]


class Camera(ctypes.Structure):
    _fields_ = [("raster_to_camera", ctypes.c_float * 16), ("cam2world_m", ctypes.c_float * 16),
                ("lens_radius", ctypes.c_float), ("focal_distance", ctypes.c_float),
                ("shutter_open", ctypes.c_float), ("shutter_close", ctypes.c_float),
                ("xres", ctypes.c_int32), ("yres", ctypes.c_int32),
                ("px_start", ctypes.c_int32), ("px_count", ctypes.c_int32),
                ("py_start", ctypes.c_int32), ("py_count", ctypes.c_int32),
                ("sx_start", ctypes.c_int32), ("sx_end", ctypes.c_int32),
                ("sy_start", ctypes.c_int32), ("sy_end", ctypes.c_int32),
                ("dx_camera", ctypes.c_float * 3), ("dy_camera", ctypes.c_float * 3), ("ortho", ctypes.c_int32),
                ("pad", ctypes.c_int32)]


P = ctypes.c_void_p
I32 = ctypes.c_int32


class Lens(ctypes.Structure):
    _fields_ = [("n_elements", I32), ("chromatic", I32), ("film_distance", ctypes.c_float),
                ("film_diag", ctypes.c_float), ("curve_radius", ctypes.c_float),
                ("aperture_offset", ctypes.c_float * 2), ("film_center", ctypes.c_float * 2),
                ("pinhole_exit", ctypes.c_float * 3), ("focal_length", ctypes.c_float), ("fstop", ctypes.c_float),
                ("diffraction", I32), ("reserved", I32), ("elements", P),
                ("num_pinholes_w", I32), ("num_pinholes_h", I32), ("microlens", I32), ("ior_eye", I32),
                ("pinholes", P), ("eye_ior", P)]


class FlatScene(ctypes.Structure):
    _fields_ = [("abi_version", I32), ("n_bands", I32), ("max_depth", I32), ("spp", I32),
                ("seed", ctypes.c_uint32), ("y_int", ctypes.c_float), ("band_Y", P),
                ("camera", Camera),
                ("n_nodes", I32), ("nodes", P), ("n_prims", I32), ("prims", P),
                ("n_tris", I32), ("tris", P), ("n_meshes", I32), ("meshes", P),
                ("n_verts", I32), ("vert_p", P), ("vert_n", P), ("vert_uv", P),
                ("n_quadrics", I32), ("quadrics", P), ("n_materials", I32), ("materials", P),
                ("n_lights", I32), ("lights", P), ("n_light_shapes", I32), ("light_shapes", P),
                ("n_spectra_floats", I32), ("spectra", P),
                ("n_instances", I32), ("instances", P), ("prim_instance", P),
                ("n_kdnodes", I32), ("kdnodes", P),
                ("n_textures", I32), ("textures", P), ("ewa_lut", P), ("rgb_basis", P),
                ("n_merl_floats", I32), ("merl", P), ("integrator", I32), ("dl_strategy", I32),
                ("meta_strategy", I32), ("prim_meta", P), ("renderer", I32), ("wave_bands", I32),
                ("spectral_sampling", I32), ("camera_type", I32), ("lens", Lens),
                ("n_texel_floats", I32), ("texels", P), ("camera_motion", P)]


PBRTHOST_ABI_VERSION = 2   # include/pbrthost.h


class Overrides(ctypes.Structure):
    _fields_ = [("abi_version", I32), ("xres", I32), ("yres", I32), ("spp", I32), ("maxdepth", I32), ("bands", I32),
                ("seed", ctypes.c_uint32), ("integrator", I32), ("dl_strategy", I32), ("meta_strategy", I32),
                ("renderer", I32), ("wave_bands", I32), ("spectral_sampling", I32)]


INTEGRATORS = {"path": 0, "directlighting": 1, "metadata": 2}
DL_STRATEGIES = {"all": 0, "one": 1}
META_STRATEGIES = {"mesh": 0, "material": 1, "depth": 2}
RENDERERS = {"sampler": 0, "spectral": 1}
SPECTRAL_SAMPLING = {"single": 0, "sampler": 1}   # samplingMethod singleDirection / samplerDirection


class RenderDesc(ctypes.Structure):
    _fields_ = [("spp_begin", I32), ("spp_end", I32), ("tile_w", I32), ("tile_h", I32),
                ("flags", I32), ("reserved", I32 * 3)]


STAT_PATHS, STAT_KERNEL_MS, STAT_ACCUM_MS, STAT_ZEROED, STAT_SPILLS, STAT_PASSES = 0, 1, 2, 3, 4, 5
F_ACCUMULATE, F_COUNT_WORK = 1, 2
KEEP_SEED = 0xFFFFFFFF
ABI_VERSION = 16


class Timing(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double * 4), ("launches", I32 * 4), ("passes", I32), ("shade_feat", I32),
                ("work", ctypes.c_uint64 * 12)]
    KERNELS = ("k_trace_closest", "k_trace_shadow", "k_shade", "k_accum")
    WORK = ("rays", "shadow_rays", "nodes_closest", "nodes_shadow", "tris_closest", "tris_shadow", "quads_closest",
            "quads_shadow", "hits", "mis_rays", "mis_hits")

_host = None
_gpu = None


def _load(name):
    path = os.path.join(LIBDIR, name)
    if name == "libpbrtgpu.so" and os.environ.get("PBRTGPU_LIB"):   # timing experiments only
        path = os.environ["PBRTGPU_LIB"]
    if not os.path.exists(path):
        raise RuntimeError("%s not built (run __graft_entry__.build() or make -C pbrt-v2-spectral_amd)" % path)
    return ctypes.CDLL(path)


def host_lib():
    global _host
    if _host is None:
        _host = _load("libpbrthost.so")
        if _host.pbrthost_abi_version() != PBRTHOST_ABI_VERSION:
            raise RuntimeError("libpbrthost.so ABI %d, this mirror expects %d" % (_host.pbrthost_abi_version(),
                                                                                 PBRTHOST_ABI_VERSION))
        _host.pbrthost_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(Overrides), ctypes.POINTER(P),
                                        ctypes.c_char_p, ctypes.c_int]
        _host.pbrthost_flat.argtypes = [P, ctypes.POINTER(FlatScene)]
        _host.pbrthost_free.argtypes = [P]
        _host.pbrthost_save_pack.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        _host.pbrthost_set_render.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        _host.pbrthost_info.argtypes = [P, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
        _host.pbrthost_write_dat.argtypes = [ctypes.c_char_p, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _host.pbrthost_write_dat_scene.argtypes = [P, ctypes.c_char_p, P, P]
        _host.pbrthost_spectrum_from_rgb.argtypes = [ctypes.c_int, P, ctypes.c_int, P]
        _host.pbrthost_write_metadata.argtypes = [P, ctypes.c_char_p]
        _host.pbrthost_set_loop_subdivider.argtypes = [P, P]
        _host.pbrthost_loop_refine.argtypes = [I32, I32, P, P, I32, P, P, P, P]
    return _host


def host_symbols():
    """Symbols declared in include/pbrthost.h."""
    return ["pbrthost_abi_version", "pbrthost_load", "pbrthost_free", "pbrthost_flat", "pbrthost_save_pack", "pbrthost_set_render",
            "pbrthost_info", "pbrthost_write_dat", "pbrthost_write_dat_scene", "pbrthost_spectrum_from_rgb",
            "pbrthost_write_metadata", "pbrthost_set_loop_subdivider", "pbrthost_loop_refine"]


def _loop_call(fn, vi, P, levels, *lead):
    """Run a subdivider with the pbrthost_loop_subdivider convention -> (P, N, vi)."""
    vi = np.ascontiguousarray(vi, np.int32).reshape(-1, 3)
    P = np.ascontiguousarray(P, np.float32).reshape(-1, 3)
    nv = np.zeros(1, np.int32)
    rc = fn(*lead, len(vi), len(P), vi.ctypes.data, P.ctypes.data, levels, nv.ctypes.data, None, None, None)
    if rc != 0:
        raise RuntimeError("loop subdivision failed (%d)" % rc)
    Po, No = np.zeros((nv[0], 3), np.float32), np.zeros((nv[0], 3), np.float32)
    vo = np.zeros((len(vi) << (2 * levels), 3), np.int32)
    rc = fn(*lead, len(vi), len(P), vi.ctypes.data, P.ctypes.data, levels, nv.ctypes.data, Po.ctypes.data,
            No.ctypes.data, vo.ctypes.data)
    if rc != 0:
        raise RuntimeError("loop subdivision failed (%d)" % rc)
    return Po, No, vo


def loop_refine_host(vi, P, levels):
    """The front end's LoopSubdiv::Refine of a control mesh (object space): (P, N, vi)."""
    return _loop_call(host_lib().pbrthost_loop_refine, vi, P, levels)


def use_gpu_subdivision(device):
    """Scenes loaded from now on refine their loopsubdiv shapes on `device` (a Device), or on
    the host again with None (pbrthost_set_loop_subdivider + pbrtgpu_loop_subdivide_hook)."""
    if device is None:
        host_lib().pbrthost_set_loop_subdivider(None, None)
    else:
        fn = ctypes.cast(gpu_lib().pbrtgpu_loop_subdivide_hook, P)
        host_lib().pbrthost_set_loop_subdivider(fn, device.ctx)


def spectrum_from_rgb(rgb, bands=32, illuminant=False):
    """SampledSpectrum::FromRGB (spectrum.cpp:93-178) as restated by the host front end."""
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    out = np.zeros(bands, dtype=np.float32)
    if host_lib().pbrthost_spectrum_from_rgb(bands, rgb.ctypes.data, 1 if illuminant else 0, out.ctypes.data) != 0:
        raise ValueError("unsupported band count %d" % bands)
    return out


def gpu_lib():
    """The product library. Raises if it is missing -- no silent fallback."""
    global _gpu
    if _gpu is None:
        _gpu = _load("libpbrtgpu.so")
        g = _gpu
        g.pbrtgpu_last_error.restype = ctypes.c_char_p
        g.pbrtgpu_context_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        g.pbrtgpu_context_destroy.argtypes = [P]
        g.pbrtgpu_scene_upload.argtypes = [P, ctypes.POINTER(FlatScene)]
        g.pbrtgpu_render_tiles.argtypes = [P, ctypes.POINTER(RenderDesc), P, I32, P]
        g.pbrtgpu_film_read.argtypes = [P, P, ctypes.c_int64]
        g.pbrtgpu_film_clear.argtypes = [P]
        g.pbrtgpu_trace_paths.argtypes = [P, P, I32, P]
        g.pbrtgpu_intersect.argtypes = [P, P, I32, P, P]
        if hasattr(g, "pbrtgpu_mt_sequence"):   # (experiment libraries of earlier builds lack it)
            g.pbrtgpu_mt_sequence.argtypes = [P, ctypes.c_uint32, I32, P]
        g.pbrtgpu_path_stats.argtypes = [P, P, I32, P]
        g.pbrtgpu_last_timing.argtypes = [P, ctypes.POINTER(Timing)]
        g.pbrtgpu_film_gather.argtypes = [P, I32, I32, P, I32, P, ctypes.c_int64]
        g.pbrtgpu_render_multi.argtypes = [P, I32, ctypes.POINTER(RenderDesc), P, I32, I32, P, ctypes.c_int64, P]
        g.pbrtgpu_build_bvh.argtypes = [P, I32, P, P, P, P]
        g.pbrtgpu_loop_subdivide.argtypes = [P, I32, I32, P, P, I32, P, P, P, P, P]
        g.pbrtgpu_loop_subdivide_hook.argtypes = [P, I32, I32, P, P, I32, P, P, P, P]
        g.pbrtgpu_libmf_eval.argtypes = [P, I32, ctypes.c_int64, P, P, P]
    return _gpu


def gpu_symbols():
    """Symbols declared in include/pbrtgpu.h (checked by the CPU test suite)."""
    return ["pbrtgpu_abi_version", "pbrtgpu_device_count", "pbrtgpu_context_create",
            "pbrtgpu_context_destroy", "pbrtgpu_last_error", "pbrtgpu_scene_upload",
            "pbrtgpu_render_tiles", "pbrtgpu_film_read", "pbrtgpu_film_clear",
            "pbrtgpu_trace_paths", "pbrtgpu_intersect", "pbrtgpu_mt_sequence", "pbrtgpu_path_stats", "pbrtgpu_last_timing",
            "pbrtgpu_film_gather", "pbrtgpu_render_multi", "pbrtgpu_build_bvh", "pbrtgpu_loop_subdivide",
            "pbrtgpu_loop_subdivide_hook", "pbrtgpu_libmf_eval"]


def tile_grid(scene, tile=16):
    """(ntx, nty) of the film-pixel tile grid the C ABI uses (pbrtgpu.h, pbrtgpu_render_desc)."""
    tw, th = (tile, tile) if isinstance(tile, int) else tile
    return (scene.width + tw - 1) // tw, (scene.height + th - 1) // th


def tile_slice(ntiles, j, m):
    """Slice j of m of a frame's tiles: tiles j, j + m, j + 2m, ... (interleaved, so every
    slice spreads over the whole image and slices cost about the same).  The same dealing as
    pbrtgpu_render_multi; a rank of a multi-process render takes slice `rank` of `world`."""
    return np.arange(j, ntiles, m, dtype=np.int32)


class Scene:
    """A flattened scene (host-owned arrays), from a .pbrt file or a .pack scene pack."""

    def __init__(self, handle):
        self._h = handle
        self.flat = FlatScene()
        host_lib().pbrthost_flat(self._h, ctypes.byref(self.flat))

    @staticmethod
    def load(path, xres=-1, yres=-1, spp=-1, maxdepth=-1, bands=0, seed=None, integrator=None, strategy=None,
             renderer=None, wave_bands=0, sampling=None):
        """bands <= 0: the pack's own band count, or 32 (the reference build) for a .pbrt file.
        integrator / strategy: None keeps the scene's SurfaceIntegrator ("path",
        "directlighting" or "metadata") and its "strategy" (DirectLighting "all" / "one",
        metadata "mesh" / "material" / "depth").  renderer ("sampler" / "spectral"),
        wave_bands and sampling ("single" / "sampler"): None / 0 keep the scene's Renderer
        and its "nWaveBands" / "samplingMethod"."""
        h = P()
        err = ctypes.create_string_buffer(1024)
        ov = Overrides(PBRTHOST_ABI_VERSION, xres, yres, spp, maxdepth, bands, KEEP_SEED if seed is None else seed,
                       -1 if integrator is None else INTEGRATORS[integrator],
                       DL_STRATEGIES.get(strategy, -1), META_STRATEGIES.get(strategy, -1),
                       -1 if renderer is None else RENDERERS[renderer], wave_bands,
                       -1 if sampling is None else SPECTRAL_SAMPLING[sampling])
        if strategy is not None and strategy not in DL_STRATEGIES and strategy not in META_STRATEGIES:
            raise ValueError("unknown strategy %r" % strategy)
        if host_lib().pbrthost_load(path.encode(), ctypes.byref(ov), ctypes.byref(h), err, 1024) != 0:
            raise RuntimeError("scene load failed: %s" % err.value.decode())
        return Scene(h)

    def paths_per_sample(self):
        """paths traced per camera sample: nWaveBands for the SpectralRenderer's
        singleDirection method, else 1"""
        f = self.flat
        return f.wave_bands if f.renderer == RENDERERS["spectral"] and f.spectral_sampling == 0 else 1

    def set_render(self, spp=-1, maxdepth=-1, seed=0):
        host_lib().pbrthost_set_render(self._h, spp, maxdepth, seed)
        host_lib().pbrthost_flat(self._h, ctypes.byref(self.flat))

    def save_pack(self, path):
        err = ctypes.create_string_buffer(1024)
        if host_lib().pbrthost_save_pack(self._h, path.encode(), err, 1024) != 0:
            raise RuntimeError(err.value.decode())

    def info(self):
        a = (ctypes.c_int64 * 16)()
        host_lib().pbrthost_info(self._h, a, 16)
        keys = ["bands", "spp", "maxdepth", "nodes", "prims", "tris", "meshes", "verts", "quadrics",
                "materials", "lights", "bvh_depth", "width", "height", "warnings"]
        return dict(zip(keys, list(a)))

    @property
    def bands(self):
        return self.flat.n_bands

    @property
    def width(self):
        return self.flat.camera.px_count

    @property
    def height(self):
        return self.flat.camera.py_count

    @property
    def spp(self):
        return self.flat.spp

    def write_metadata(self, image_file):
        """pbrtWorldEnd's _mesh.txt / _materials.txt beside image_file; True if one was written."""
        r = host_lib().pbrthost_write_metadata(self._h, image_file.encode())
        if r < 0:
            raise RuntimeError("cannot write metadata for %s" % image_file)
        return r == 1

    def prim_meta(self):
        """[n_prims][2] uint32: the primitiveId / materialId a hit on each primitive reports."""
        n = self.flat.n_prims
        if not self.flat.prim_meta:
            return np.zeros((n, 2), np.uint32)
        buf = (ctypes.c_uint32 * (2 * n)).from_address(self.flat.prim_meta)
        return np.frombuffer(buf, dtype=np.uint32).reshape(n, 2).copy()

    def write_dat(self, path, film):
        film = np.ascontiguousarray(film, dtype=np.float32)
        assert film.shape == (self.height, self.width, self.bands)
        if host_lib().pbrthost_write_dat_scene(self._h, path.encode(), film.ctypes.data, None) != 0:
            raise RuntimeError("cannot write %s" % path)

    def __del__(self):
        try:
            if self._h:
                host_lib().pbrthost_free(self._h)
        except Exception:
            pass


def _arr(ptr, ctype, n):
    return np.frombuffer((ctype * n).from_address(ptr), dtype=np.dtype(ctype)).copy() if n else np.zeros(0, np.dtype(ctype))


def prim_bounds(scene):
    """[n_prims][6] float32 world bounds of the scene's primitives (bmin, bmax): a triangle's
    three world-space vertices (Triangle::WorldBound, trianglemesh.cpp:97-103); a sphere's, disk's
    or cylinder's object bound (sphere.cpp:42-46, disk.cpp:41-45, cylinder.cpp:40-44) through ObjectToWorld's eight corners
    (transform.cpp:144-156), evaluated in double and rounded outward to float.  The input of
    the GPU BVH build (pbrtgpu_build_bvh)."""
    f = scene.flat
    if f.n_instances:
        raise ValueError("the GPU BVH build covers scenes without instances")
    n = f.n_prims
    prims = _arr(f.prims, ctypes.c_int32, 4 * n).reshape(n, 4)
    out = np.zeros((n, 6), np.float32)
    tri = prims[:, 0] == SHAPE_TRIANGLE
    if tri.any():
        tv = _arr(f.tris, ctypes.c_int32, 4 * f.n_tris).reshape(-1, 4)[:, 1:]
        vp = _arr(f.vert_p, ctypes.c_float, 3 * f.n_verts).reshape(-1, 3)
        pts = vp[tv[prims[tri, 1]]]                      # [k][3 vertices][xyz]
        out[tri, :3] = pts.min(axis=1)
        out[tri, 3:] = pts.max(axis=1)
    quads = np.nonzero(~tri)[0]
    if len(quads):
        q = _arr(f.quadrics, ctypes.c_float, 44 * f.n_quadrics).reshape(-1, 44)
        qt = q[:, 0].view(np.int32)
        for i in quads:
            r = q[prims[i, 1]]
            rad, zmin, zmax, h = float(r[36]), float(r[37]), float(r[38]), float(r[42])
            if qt[prims[i, 1]] in (SHAPE_SPHERE, SHAPE_CYLINDER):   # cylinder.cpp:40-44
                lo, hi = (-rad, -rad, zmin), (rad, rad, zmax)
            else:
                lo, hi = (-rad, -rad, h), (rad, rad, h)
            m = r[4:20].astype(np.float64).reshape(4, 4)
            c = np.array([[x, y, z, 1.0] for x in (lo[0], hi[0]) for y in (lo[1], hi[1]) for z in (lo[2], hi[2])])
            w = c @ m.T
            p = w[:, :3] / np.where(w[:, 3:] == 1.0, 1.0, w[:, 3:])
            out[i, :3] = np.nextafter(p.min(axis=0).astype(np.float32), np.float32(-np.inf))
            out[i, 3:] = np.nextafter(p.max(axis=0).astype(np.float32), np.float32(np.inf))
    return out


class BvhScene(Scene):
    """A scene over a BVH built on the GPU (pbrtgpu_build_bvh): the parent's flattened scene
    with new nodes and its per-primitive arrays (prims, prim_instance, prim_meta) permuted
    into the new leaf order.  Everything else is shared with the parent."""

    def __init__(self, parent, nodes, order, build_ms):
        self.parent = parent
        self._h = parent._h
        self.build_ms = build_ms
        self.order = order
        self.flat = FlatScene.from_buffer_copy(parent.flat)
        f, n = parent.flat, parent.flat.n_prims
        self._nodes = nodes
        self._prims = np.ascontiguousarray(_arr(f.prims, ctypes.c_int32, 4 * n).reshape(n, 4)[order])
        self.flat.n_nodes, self.flat.nodes = len(nodes), nodes.ctypes.data
        self.flat.prims = self._prims.ctypes.data
        if f.prim_instance:
            self._pi = np.ascontiguousarray(_arr(f.prim_instance, ctypes.c_int32, n)[order])
            self.flat.prim_instance = self._pi.ctypes.data
        if f.prim_meta:
            self._pm = np.ascontiguousarray(_arr(f.prim_meta, ctypes.c_uint32, 2 * n).reshape(n, 2)[order])
            self.flat.prim_meta = self._pm.ctypes.data

    def __del__(self):
        pass   # the parent owns the host scene


def _check(rc):
    if rc != 0:
        msg = gpu_lib().pbrtgpu_last_error()
        raise RuntimeError("pbrtgpu error %d: %s" % (rc, msg.decode() if msg else "?"))


class Device:
    """One pbrtgpu context on one GPU (one host thread drives it)."""

    def __init__(self, device=0):
        self.lib = gpu_lib()
        self.ctx = P()
        _check(self.lib.pbrtgpu_context_create(device, ctypes.byref(self.ctx)))
        self.scene = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def close(self):
        if self.ctx:
            self.lib.pbrtgpu_context_destroy(self.ctx)
            self.ctx = P()

    def upload(self, scene):
        _check(self.lib.pbrtgpu_scene_upload(self.ctx, ctypes.byref(scene.flat)))
        self.scene = scene

    def build_bvh(self, scene):
        """The scene over a BVH built on this GPU (pbrtgpu_build_bvh) -> BvhScene with
        build_ms = (device ms, call wall ms).  Needs no uploaded scene."""
        b = prim_bounds(scene)
        n = len(b)
        nodes = np.zeros(2 * n - 1, dtype=np.dtype([("bmin", "<f4", 3), ("bmax", "<f4", 3), ("offset", "<u4"),
                                                     ("meta", "<u4")]))
        order = np.zeros(n, np.int32)
        ms = np.zeros(2, np.float64)
        rc = self.lib.pbrtgpu_build_bvh(self.ctx, n, b.ctypes.data, nodes.ctypes.data, order.ctypes.data, ms.ctypes.data)
        if rc < 0:
            _check(rc)
        assert rc == 2 * n - 1
        return BvhScene(scene, nodes, order, (float(ms[0]), float(ms[1])))

    def loop_subdivide(self, vi, P, levels):
        """Loop subdivision of a control mesh on this GPU (pbrtgpu_loop_subdivide): (P, N, vi)."""
        return _loop_call(self.lib.pbrtgpu_loop_subdivide_hook, vi, P, levels, self.ctx)

    def render(self, spp_begin=0, spp_end=None, tiles=None, tile=(16, 16), accumulate=False, stats=None,
               count_work=False):
        s = self.scene
        desc = RenderDesc(spp_begin, s.spp if spp_end is None else spp_end, tile[0], tile[1],
                          (F_ACCUMULATE if accumulate else 0) | (F_COUNT_WORK if count_work else 0), (I32 * 3)())
        st = np.zeros(8, dtype=np.float64)
        if tiles is None:
            _check(self.lib.pbrtgpu_render_tiles(self.ctx, ctypes.byref(desc), None, 0, st.ctypes.data))
        else:
            t = np.ascontiguousarray(tiles, dtype=np.int32)
            _check(self.lib.pbrtgpu_render_tiles(self.ctx, ctypes.byref(desc), t.ctypes.data, len(t),
                                                 st.ctypes.data))
        if stats is not None:
            stats[:] = st
        return st

    def film(self):
        s = self.scene
        out = np.zeros((s.height, s.width, s.bands), dtype=np.float32)
        _check(self.lib.pbrtgpu_film_read(self.ctx, out.ctypes.data, out.size))
        return out

    def gather(self, out, tiles=None, tile=(16, 16)):
        """Host gather: writes the film pixels of `tiles` (all when None) into `out` (a float32
        [H][W][bands] array, e.g. a shared-memory film), leaving its other pixels untouched."""
        s = self.scene
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.size >= s.height * s.width * s.bands
        if tiles is None:
            _check(self.lib.pbrtgpu_film_gather(self.ctx, tile[0], tile[1], None, 0, out.ctypes.data, out.size))
        else:
            t = np.ascontiguousarray(tiles, dtype=np.int32)
            _check(self.lib.pbrtgpu_film_gather(self.ctx, tile[0], tile[1], t.ctypes.data, len(t), out.ctypes.data,
                                                out.size))
        return out

    def clear(self):
        _check(self.lib.pbrtgpu_film_clear(self.ctx))

    def trace_paths(self, keys):
        keys = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        out = np.zeros((len(keys), self.scene.bands), dtype=np.float32)
        _check(self.lib.pbrtgpu_trace_paths(self.ctx, keys.ctypes.data, len(keys), out.ctypes.data))
        return out

    def mt_sequence(self, seed, n):
        """The first n outputs of RNG(seed) as the shading kernels draw them (pbrtgpu_mt_sequence)."""
        out = np.zeros(n, np.uint32)
        _check(self.lib.pbrtgpu_mt_sequence(self.ctx, seed, n, out.ctypes.data))
        return out

    def libmf_eval(self, fn, x, y=None):
        """The shading kernels' float transcendental `fn` (a LIBMF name) over x (and y for powf /
        atan2f) on this GPU (pbrtgpu_libmf_eval); sincosf returns [n][2] (sin, cos)."""
        return _libmf_call(lambda f, n, xp, yp, op: _check(self.lib.pbrtgpu_libmf_eval(self.ctx, f, n, xp, yp, op)),
                           fn, x, y)

    def intersect(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros((len(rays), 4), dtype=np.float32)
        occ = np.zeros(len(rays), dtype=np.int32)
        _check(self.lib.pbrtgpu_intersect(self.ctx, rays.ctypes.data, len(rays), hits.ctypes.data,
                                          occ.ctypes.data))
        return hits, occ

    def path_stats(self, keys):
        """Traversal work counters: rays, shadow rays, nodes, triangle tests, quadric tests, hits."""
        keys = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        out = np.zeros(6, dtype=np.uint64)
        _check(self.lib.pbrtgpu_path_stats(self.ctx, keys.ctypes.data, len(keys), out.ctypes.data))
        return dict(zip(["rays", "shadow_rays", "nodes", "tri_tests", "quad_tests", "hits"], [int(v) for v in out]))

    def timing(self):
        """Per-kernel device ms / launches of the last call, passes, and work counters."""
        t = Timing()
        _check(self.lib.pbrtgpu_last_timing(self.ctx, ctypes.byref(t)))
        out = {"passes": t.passes, "shade_feat": t.shade_feat}
        for i, k in enumerate(Timing.KERNELS):
            out[k] = {"ms": t.ms[i], "launches": t.launches[i]}
        out["work"] = {k: int(t.work[i]) for i, k in enumerate(Timing.WORK)}
        return out


# float transcendentals of include/pbrt_libmf.h (PBRTGPU_LIBMF_* order)
LIBMF = ["sinf", "cosf", "sincosf", "expf", "logf", "acosf", "atanf", "tanf", "powf", "atan2f"]


def _libmf_call(call, fn, x, y):
    f = LIBMF.index(fn)
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    yp = None
    if fn in ("powf", "atan2f"):
        y = np.ascontiguousarray(y, dtype=np.float32).ravel()
        assert len(y) == len(x)
        yp = y.ctypes.data
    out = np.zeros(2 * len(x) if fn == "sincosf" else len(x), np.float32)
    call(f, len(x), x.ctypes.data, yp, out.ctypes.data)
    return out.reshape(-1, 2) if fn == "sincosf" else out


def render_multi(devices, spp_begin=0, spp_end=None, tiles=None, tile=(16, 16), slices_per_device=1, out=None,
                 accumulate=False):
    """One frame over several Devices (one per GPU, same scene uploaded): pbrtgpu_render_multi
    -- one host thread per device pulls interleaved tile slices, then gathers its tiles into
    the returned film.  Returns (film, per-device stats [n][8])."""
    s = devices[0].scene
    n = len(devices)
    arr = (P * n)(*[d.ctx for d in devices])
    desc = RenderDesc(spp_begin, s.spp if spp_end is None else spp_end, tile[0], tile[1],
                      F_ACCUMULATE if accumulate else 0, (I32 * 3)())
    if out is None:
        out = np.zeros((s.height, s.width, s.bands), dtype=np.float32)
    st = np.zeros((n, 8), dtype=np.float64)
    if tiles is None:
        tp, nt = None, 0
    else:
        t = np.ascontiguousarray(tiles, dtype=np.int32)
        tp, nt = t.ctypes.data, len(t)
    _check(gpu_lib().pbrtgpu_render_multi(arr, n, ctypes.byref(desc), tp, nt, slices_per_device, out.ctypes.data,
                                          out.size, st.ctypes.data))
    return out, st


# ---------------------------------------------------------------- test infrastructure
class Oracle:
    """CPU restatement (oracle/liboracle*.so). TEST INFRASTRUCTURE ONLY."""

    def __init__(self, libm_float=False):
        name = "liboracle_libm.so" if libm_float else "liboracle.so"
        path = os.path.join(ROOT, "oracle", name)
        if not os.path.exists(path):
            raise RuntimeError("%s not built (make -C oracle)" % path)
        self.lib = ctypes.CDLL(path)
        self.lib.oracle_trace_paths.argtypes = [ctypes.POINTER(FlatScene), P, I32, P]
        self.lib.oracle_intersect.argtypes = [ctypes.POINTER(FlatScene), P, I32, P, P]
        self.lib.oracle_render.argtypes = [ctypes.POINTER(FlatScene), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, P, ctypes.c_int, P]
        self.lib.oracle_trace_range.argtypes = [ctypes.POINTER(FlatScene), ctypes.c_long, ctypes.c_long,
                                                ctypes.c_int]
        self.lib.oracle_trace_range.restype = ctypes.c_long
        self.lib.oracle_mt_first.argtypes = [ctypes.c_uint32, ctypes.c_int, P]
        self.lib.oracle_libmf_eval.argtypes = [ctypes.c_int, ctypes.c_int64, P, P, P]

    def mt_first(self, seed, n):
        out = np.zeros(n, dtype=np.uint32)
        self.lib.oracle_mt_first(seed, n, out.ctypes.data)
        return out

    def libmf_eval(self, fn, x, y=None):
        """this build's float transcendental `fn` (glibc's in the libm build, the restatement
        include/pbrt_libmf.h otherwise)"""
        def call(f, n, xp, yp, op):
            if self.lib.oracle_libmf_eval(f, n, xp, yp, op) != 0:
                raise ValueError(fn)
        return _libmf_call(call, fn, x, y)

    def trace_paths(self, scene, keys):
        keys = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 3)
        out = np.zeros((len(keys), scene.bands), dtype=np.float32)
        self.lib.oracle_trace_paths(ctypes.byref(scene.flat), keys.ctypes.data, len(keys), out.ctypes.data)
        return out

    def intersect(self, scene, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        hits = np.zeros((len(rays), 4), dtype=np.float32)
        occ = np.zeros(len(rays), dtype=np.int32)
        self.lib.oracle_intersect(ctypes.byref(scene.flat), rays.ctypes.data, len(rays), hits.ctypes.data,
                                  occ.ctypes.data)
        return hits, occ

    def render(self, scene, window=None, threads=8):
        c = scene.flat.camera
        x0, x1, y0, y1 = window if window is not None else (c.sx_start, c.sx_end, c.sy_start, c.sy_end)
        film = np.zeros((scene.height, scene.width, scene.bands), dtype=np.float32)
        st = np.zeros(4, dtype=np.float64)
        self.lib.oracle_render(ctypes.byref(scene.flat), x0, x1, y0, y1, film.ctypes.data, threads, st.ctypes.data)
        return film, st

    def trace_range(self, scene, first, count, threads):
        return self.lib.oracle_trace_range(ctypes.byref(scene.flat), first, count, threads)


def oracle(libm_float=False):
    return Oracle(libm_float)
