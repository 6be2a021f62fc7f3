"""bench.py -- Mpaths/s of the MI355X spectral path tracer on BASELINE.json's configs.

Workload (default --config c2 = BASELINE.json configs[1], the metric's configuration):
killeroo-simple, SampledSpectrum 32 bands (the reference build's nSpectralSamples;
BASELINE's "30 bands" names the same config), 'path' integrator maxdepth 5, 700x700 film,
256 spp -> 125.44 M camera paths per step.  --config c3 | c4 | c5 runs the other packaged
configs at their stated sizes (bunny 1920x1080@1024 measured BRDF; metal 400x400@4096 60 bands;
anim-killeroos-moving 600x600@512 motion blur).

One step = one frame: every camera path traced, every sample added to the film in the
reference's order, and the film back on the host (first kernel launch ->
film tiles on the host).  The scene is uploaded once before timing, so inputs are resident
in HBM when the timed region starts.

Multi-GPU: ONE frame's 16x16 film-pixel tiles are dealt into interleaved
slices (pbrtgpu.tile_slice), one per GPU; every GPU renders its slice and gathers its pixels
into one host film (pbrtgpu_film_gather).  Nothing is exchanged between GPUs (no RCCL).
  * python -m torch.distributed.run --nproc-per-node N bench.py --gpus N: one process per
    GPU (LOCAL_RANK); the film is a shared-memory file every rank writes its own pixels into;
    the barrier around the timed region and the max over ranks of the elapsed time go over
    gloo (host only).  value = the frame's paths x steps / max elapsed ("strong": the total
    work of a step is one frame whatever N is).
  * python bench.py --gpus N (no launcher): one process, N contexts, one host thread each
    (pbrtgpu_render_multi).
--shard frames instead gives every rank its own frame (seed = rank; "weak").

Extra JSON fields:
  roofline     the dominant kernel's algorithmic bytes per launch / its EXCLUSIVE average
               launch time, from one untimed frame in serial mode (PBRTGPU_SERIAL=1: one
               lane, no concurrent kernels, so each kernel's HIP-event spans are its own
               device time); per-kernel table beside it (ms, GB/s, frac, PMC traffic from
               profiles/hbm_traffic.json when it holds this config).  DESIGN.md §5.
  cpu_baseline the CPU restatement (oracle/liboracle_libm.so, TEST INFRASTRUCTURE) timed on this
               host: every core this process may use, and one core, over a bounded sample of
               the same frame (all spp of pseudo-randomly spread pixels).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md "HBM [CDNA4]": 8 TB/s peak
NODE_BYTES, TRI_BYTES, QUAD_BYTES = 32, 48, 176
RAY_BYTES, HIT_BYTES, QENTRY_BYTES = 36, 8, 4     # SoA ray record read, hit / occlusion written, queue entry
METRIC = "Mpaths/sec (whole node) + HBM GB/s; spectral path tracer at 1/2/4/8 MI355X"

# BASELINE.json configs -> scene packs (built from the reference's scene files with SURVEY.md
# App. B overrides: 'path' integrator maxdepth 5, lowdiscrepancy spp, resolution, bands)
CONFIGS = {
    "c1": ("killeroo-simple-rgb.pack", "killeroo-simple RGBSpectrum (%d channels), path maxdepth %d, %dspp, %dx%d"),
    "c2": ("killeroo-simple.pack", "killeroo-simple SampledSpectrum %d bands, path maxdepth %d, %dspp, %dx%d"),
    "c3": ("bunny.pack", "bunny (mystique measured BRDF) SampledSpectrum %d bands, path maxdepth %d, %dspp, %dx%d"),
    "c4": ("metal.pack", "metal (Au conductor, env light) SampledSpectrum %d bands, path maxdepth %d, %dspp, %dx%d"),
    # not a BASELINE config: C2's scene in the 60-band build (the plain 60-band kernels, e.g. DirectLighting)
    "c2_b60": ("killeroo-simple-b60.pack", "killeroo-simple SampledSpectrum %d bands, path maxdepth %d, %dspp, %dx%d"),
    "c5": ("anim-killeroos-moving.pack",
           "anim-killeroos-moving (motion-blur BVHs) SampledSpectrum %d bands, path maxdepth %d, %dspp, %dx%d"),
}


NODE4_BYTES = 128              # a node of the shadow queries' 4-wide BVH copy (4 child boxes + refs)
NODE4Q_BYTES = 64              # a node of its quantized copy (k_trace_s4q: 8-bit child boxes + refs)


def wide4_active(scene, kind):
    """the closest-hit / shadow queries run on the 4-wide BVH copy (k_trace_c4 / k_trace_s4):
    scenes without instances, unless PBRTGPU_CLOSEST4=0 / PBRTGPU_SHADOW4=0"""
    var = "PBRTGPU_CLOSEST4" if kind == "closest" else "PBRTGPU_SHADOW4"
    return scene.flat.n_instances == 0 and os.environ.get(var, "1") != "0"


def shadow4q_active(scene):
    """the shadow queries run on the quantized 4-wide copy (k_trace_s4q) with PBRTGPU_SHADOW4Q=1"""
    return wide4_active(scene, "shadow") and os.environ.get("PBRTGPU_SHADOW4Q", "0") != "0"


def trace_bytes(work, kernel, wide4=False, quant=False):
    """algorithmic bytes of a traversal kernel = every BVH node it visits
    (32 B; a 4-wide node 128 B, after the root box test of 32 B per ray), every primitive
    it tests (48 B pre-gathered triangle, 176 B quadric record), plus the ray it reads, the answer
    it writes and its queue entry."""
    if kernel == "k_trace_closest":
        nodes = (NODE_BYTES * work["rays"] + NODE4_BYTES * (work["nodes_closest"] - work["rays"]) if wide4
                 else NODE_BYTES * work["nodes_closest"])
        return (nodes + TRI_BYTES * work["tris_closest"]
                + QUAD_BYTES * work["quads_closest"] + (RAY_BYTES + HIT_BYTES + QENTRY_BYTES) * work["rays"])
    nodes = (NODE_BYTES * work["shadow_rays"] + (NODE4Q_BYTES if quant else NODE4_BYTES) * (work["nodes_shadow"] - work["shadow_rays"])
             if wide4 else NODE_BYTES * work["nodes_shadow"])
    return (nodes + TRI_BYTES * work["tris_shadow"] + QUAD_BYTES * work["quads_shadow"]
            + (RAY_BYTES + 4 + QENTRY_BYTES) * work["shadow_rays"])


def shade_bytes(work, paths, bands):
    """algorithmic bytes of k_shade over a frame, from the event counts of
    the instrumented render.  S = 4*bands (one spectrum); scene gathers per vertex:
    prim 16 + triangle 16 + 3 vertices x (P 12, N 12, uv 8) + material 64 = 192 B, plus three
    BSDF-spectrum reads and one emitted-spectrum read."""
    S = 4.0 * bands
    cams = paths
    cont = work["rays"] - work["mis_rays"] - cams          # continuation rays
    verts = work["hits"] - work["mis_hits"]                # vertices shaded
    slot_state = 20.0                                      # item, hash, sample, bounce, flags
    per_vertex = slot_state * 2 + 2 * S + S + 36 + 8 + 192 + 4 * S   # L r/w, beta_b, ray, hit, scene
    per_cont = S + 36 + 4                                  # beta_{b+1}, ray, queue entry
    per_shadow = S + 36 + 4 + S                            # A write, ray, queue, A read at finish
    per_mis = S + 36 + 4 + S + 8                           # B write, ray, queue, B read, hit
    per_cam = 36 + 4 + slot_state                          # camera ray (L = 0, beta = 1 implicit)
    per_out = S
    return (verts * per_vertex + cont * per_cont + work["shadow_rays"] * per_shadow
            + work["mis_rays"] * per_mis + cams * (per_cam + per_out))


def accum_bytes(paths, bands):
    """k_accum: every per-sample radiance read once (4 B per band); film read+write per pixel
    is negligible next to it (1/spp)."""
    return 4.0 * bands * paths


def cpu_info():
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    ncpu = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else ncpu
    return model, ncpu, aff


def cgroup_cpus():
    """CPUs this process's cgroup may use (cgroup v2 cpu.max quota / period), or None"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(scene, target_s):
    """CPU restatement (oracle/liboracle_libm.so, TEST INFRASTRUCTURE: the build with glibc's float
    transcendentals, whose per-core rate profiles/cpu_calibration.json measured against the
    reference harness itself on one box) on the host: all spp of
    pseudo-randomly spread pixels of the same frame, sized to ~target_s seconds on every core
    this process may use (the affinity mask, capped by OMP_NUM_THREADS where the box sets a
    CPU share and by the cgroup's cpu.max quota: 16 CPUs of the 256-CPU host on the GPU box,
    profiles/r05/r05a/cpu_share.txt), then ~target_s / 3 on one core.  The whole host is reported
    as the one-core rate times its CPU count, marked as an extrapolation."""
    model, ncpu, aff = cpu_info()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    quota = cgroup_cpus()
    threads = max(1, min(aff, share) if share > 0 else aff)
    if quota is not None:   # more threads than the cgroup's CPU quota run no faster
        threads = max(1, min(threads, int(quota)))
    o = pg.oracle(libm_float=True)
    spp = scene.spp
    pps = scene.paths_per_sample()   # SpectralRenderer singleDirection: a sample is nWaveBands paths

    def timed(nthreads, seconds):
        probe = max(spp, 64 * spp // 16 * nthreads)
        t = time.perf_counter()
        o.trace_range(scene, 0, probe, nthreads)
        dt = time.perf_counter() - t
        count = int(max(probe, probe * seconds / max(dt, 1e-3)))
        count = (count + spp - 1) // spp * spp
        t = time.perf_counter()
        n = o.trace_range(scene, 0, count, nthreads)
        return n, time.perf_counter() - t

    n, dt = timed(threads, target_s)
    n1, dt1 = timed(1, target_s / 3.0)
    n, n1 = n * pps, n1 * pps
    per_core = n1 / dt1 / 1e6
    return {"value": round(n / dt / 1e6, 4), "unit": "Mpaths/s", "cores": threads, "kind": "port",
            "one_core": round(per_core, 4), "host_cpus": ncpu, "affinity_cpus": aff, "cpu_model": model,
            "cgroup_cpus": quota,
            "all_host_cores_extrapolated": {
                "value": round(per_core * ncpu, 2), "cores": ncpu,
                "how": "one_core x host_cpus (linear, an upper bound): this job's cgroup quota (cgroup_cpus) caps "
                       "what it can run on the host, so the whole host is not measurable from here"},
            "sample": "%d paths = all %d samples of %d pseudo-randomly spread pixels of the same frame, %.1f s on "
                      "%d threads; 1-core leg %d paths in %.1f s" % (n, spp, n // spp // pps, dt, threads, n1, dt1),
            "calibration": "this build (liboracle_libm.so) vs the reference harness per core, same box: "
                           "profiles/cpu_calibration.json (port_over_reference)"}


def reduce_over_ranks(dist, elapsed, paths, device="cpu"):
    """(max elapsed over ranks, total paths over ranks) -- host-side (gloo) reductions."""
    if dist is None:
        return elapsed, paths
    import torch
    t = torch.tensor([elapsed, paths], dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
    dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
    return float(mx[0]), float(t[1])


def one_node(world):
    """All ranks on one node (torchrun's LOCAL_WORLD_SIZE == WORLD_SIZE): the shared-memory film
    can be used.  Otherwise every rank keeps a film of its own (compose_film)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world


def compose_film(film, dist, device="cpu"):
    """Multi-node: the ranks' private films (each holding only its own tiles; the others 0) summed
    onto rank 0 over gloo -- exact, as the tile sets are disjoint.  After the timed steps only."""
    import torch
    t = torch.from_numpy(np.ascontiguousarray(film))
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
    return t.numpy()


def shared_film(shape, rank, dist, tag):
    """A host film every rank of ONE node writes its own pixels into (/dev/shm file): the host
    gather of SURVEY.md §8(e) without any collective.  Only valid when all ranks share the node
    (one_node); a /dev/shm file is invisible to other nodes."""
    path = "/dev/shm/pbrtgpu_film_%s" % tag
    n = int(np.prod(shape)) * 4
    if rank == 0:
        with open(path, "wb") as f:
            f.truncate(n)
    if dist is not None:
        dist.barrier()
    return path, np.memmap(path, dtype=np.float32, mode="r+", shape=shape)


def exclusive_roofline(dev, scene, tiles, tile, frame_paths, cfg, pps=1):
    """Per-kernel exclusive device time (serial mode) and algorithmic bytes (instrumented
    frame), both over one frame of this rank's tiles, untimed."""
    os.environ["PBRTGPU_SERIAL"] = "1"
    try:
        dev.render(tiles=tiles, tile=tile)
        tm = dev.timing()
        serial_wall = None
        t = time.perf_counter()
        dev.render(tiles=tiles, tile=tile)
        serial_wall = time.perf_counter() - t
        tm = dev.timing()
    finally:
        del os.environ["PBRTGPU_SERIAL"]
    dev.render(tiles=tiles, tile=tile, count_work=True)
    work = dev.timing()["work"]
    byts = {"k_trace_closest": trace_bytes(work, "k_trace_closest", wide4_active(scene, "closest")),
            "k_trace_shadow": trace_bytes(work, "k_trace_shadow", wide4_active(scene, "shadow"), shadow4q_active(scene)),
            "k_shade": shade_bytes(work, frame_paths, scene.bands),
            "k_accum": accum_bytes(frame_paths / pps, scene.bands)}   # one row per camera sample
    traffic = {}
    tf = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    if os.path.exists(tf):
        with open(tf) as f:
            tr = json.load(f)
        traffic = tr.get("configs", {}).get(cfg, {})
    per = {}
    for k in pg.Timing.KERNELS:
        ms, nl = tm[k]["ms"], max(tm[k]["launches"], 1)
        avg = ms / nl
        bpl = byts[k] / nl
        gbs = bpl / (avg * 1e-3) / 1e9 if avg > 0 else 0.0
        ent = traffic.get(k)
        per[k] = {"ms_per_frame": round(ms, 2), "launches": tm[k]["launches"], "avg_launch_ms": round(avg, 4),
                  "alg_bytes_per_launch": round(bpl), "alg_GBps": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                  "pmc_bytes_per_launch": ent.get("hbm_bytes_per_launch") if ent else None}
    dom = max(("k_trace_closest", "k_trace_shadow", "k_shade"), key=lambda k: per[k]["ms_per_frame"])
    d = per[dom]
    roof = {"bound": "hbm", "achieved": d["alg_GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["frac"],
            "traffic": d["pmc_bytes_per_launch"], "kernel": dom, "avg_launch_ms": d["avg_launch_ms"],
            "alg_bytes_per_launch": d["alg_bytes_per_launch"],
            "timing": "exclusive: PBRTGPU_SERIAL=1 frame (one lane, no concurrent kernels), HIP events",
            "serial_frame_ms": round(serial_wall * 1e3, 2), "kernels": per,
            "per_path": {k: round(v / frame_paths, 3) for k, v in work.items()},
            "traffic_source": (traffic.get("source") if traffic else None)}
    return roof


def slice_efficiency(dev, scene, tile, full_ms, full_paths, reps=2):
    """What one GPU does at N GPUs, on this GPU: the 1/N interleaved tile slice of the frame
    (pbrtgpu.tile_slice, as rank 0 of N renders it), rendered and gathered like a timed step,
    best of `reps`; its rate over the full-frame rate of the timed steps.  Wall time and the
    call's device time (trace + shade + accum) are both given, so the per-call fixed cost
    (host setup, spill scan, the wavefront's fill and drain) shows."""
    ntx, nty = pg.tile_grid(scene, tile)
    full_rate = full_paths / (full_ms * 1e-3)
    film = np.zeros((scene.height, scene.width, scene.bands), np.float32)
    out = {"what": "rank 0's share at N GPUs (1/N interleaved tiles) on one GPU: its Mpaths/s / the full frame's",
           "full_frame_ms": round(full_ms, 2)}
    for n in (2, 4, 8):
        tiles = pg.tile_slice(ntx * nty, 0, n)
        best, paths = None, 0.0
        for _ in range(reps + 1):   # the first call sizes the slot pools
            t = time.perf_counter()
            st = dev.render(tiles=tiles, tile=tile)
            dev.gather(film, tiles=tiles, tile=tile)
            dt = time.perf_counter() - t
            paths = st[pg.STAT_PATHS]
            best = dt if best is None else min(best, dt)
        tm = dev.timing()
        dev_ms = sum(tm[k]["ms"] for k in pg.Timing.KERNELS)
        out["1/%d" % n] = {"efficiency": round(paths / best / full_rate, 4), "ms": round(best * 1e3, 2),
                           "device_ms": round(dev_ms, 2), "passes": tm["passes"],
                           "Mpaths_s": round(paths / best / 1e6, 2)}
    return out


def setup_times(dev, scene, cfg, load_ms, upload_ms, gpu_bvh):
    """scene setup, reported apart from the timed frames (api.cpp:1309-1330 parses
    the scene and builds the accelerator before Render).  The pack load stands for the parse (the
    pack is the front end's flattened scene, SAH BVH included: pbrthost_load of a .pbrt does the
    parse, Loop subdivision and the bvh.cpp:145-194 build, which needs the reference's scene files
    that stay in the build container); the GPU BVH build (lbvh.hip) over the same primitives and
    the Loop subdivision of the killeroo control mesh (host front end and loopsubdiv.hip) are timed
    here on this box, untimed by the frames."""
    out = {"pack_load_ms": round(load_ms, 2), "upload_ms": round(upload_ms, 2),
           "what": "pack load (the front end's flattened scene incl. its SAH BVH) + pbrtgpu_scene_upload; "
                   "the GPU builds below are timed separately (not part of total_ms unless --bvh gpu)"}
    total = load_ms + upload_ms
    try:
        if not gpu_bvh:
            b = dev.build_bvh(scene)
            out["gpu_bvh_build_ms"] = {"device": round(b.build_ms[0], 3), "call": round(b.build_ms[1], 3),
                                       "prims": int(scene.flat.n_prims)}
        else:
            out["gpu_bvh_build_ms"] = {"device": round(scene.build_ms[0], 3), "call": round(scene.build_ms[1], 3)}
            total += scene.build_ms[1]
    except Exception as e:   # instanced scenes: the top level is the front end's
        out["gpu_bvh_build_ms"] = "n/a (%s)" % str(e)[:80]
    ctl = os.path.join(ROOT, "tests", "golden", "killeroo_control.npz")
    if cfg in ("c1", "c2", "c2_b60", "c5") and os.path.exists(ctl):
        g = np.load(ctl)
        vi, P, lv = g["vi"], g["P"], int(g["levels"])
        dev.loop_subdivide(vi, P, lv)   # first call: module load
        t = time.perf_counter()
        dev.loop_subdivide(vi, P, lv)
        gms = (time.perf_counter() - t) * 1e3
        t = time.perf_counter()
        pg.loop_refine_host(vi, P, lv)
        hms = (time.perf_counter() - t) * 1e3
        out["loop_subdivision_ms"] = {"gpu_call": round(gms, 3), "host_one_core": round(hms, 2), "levels": lv,
                                      "faces_in": int(len(vi))}
    out["total_ms"] = round(total, 2)
    return out


def frame_hbm(roof, cfg, integrator, renderer, step_s, n_gpus):
    """Whole-frame HBM GB/s (the metric's "+ HBM GB/s"): the PMC bytes of one frame of this workload
    (FETCH_SIZE x2 + WRITE_SIZE per kernel launch x launches, profiles/hbm_traffic.json, taken by
    tools/gpu_profile.sh on a serial-mode frame of the same tree) over this run's timed frame."""
    tf = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    if not os.path.exists(tf) or n_gpus != 1:
        return None
    key = cfg + {"path": "", "directlighting": "_dl", "metadata": "_meta"}[integrator] + (
        "" if renderer == "sampler" else "_spec")
    with open(tf) as f:
        tr = json.load(f).get("configs", {}).get(key)
    if not tr:
        return None
    byts = sum(v["hbm_bytes_per_launch"] * v["launches"] for k, v in tr.items() if isinstance(v, dict))
    out = {"bytes_per_frame": round(byts), "GBps": round(byts / step_s / 1e9, 1),
           "frac_of_peak": round(byts / step_s / 1e9 / HBM_PEAK_GBS, 4), "source": tr.get("source")}
    if roof is not None:
        alg = sum(v["alg_bytes_per_launch"] * v["launches"] for v in roof["kernels"].values())
        out["alg_bytes_per_frame"] = round(alg)
        out["alg_GBps"] = round(alg / step_s / 1e9, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--scene", default=None, help="scene pack (default: the config's)")
    ap.add_argument("--res", type=int, default=-1, help="square resolution override (default: the config's)")
    ap.add_argument("--spp", type=int, default=-1, help="spp override (default: the config's)")
    ap.add_argument("--integrator", choices=["path", "directlighting", "metadata"], default="path",
                    help="SurfaceIntegrator (BASELINE configs: path; directlighting / metadata = SURVEY §8(f) rows)")
    ap.add_argument("--strategy", choices=["all", "one", "mesh", "material", "depth"], default=None,
                    help="DirectLighting (all / one) or metadata (mesh / material / depth) strategy")
    ap.add_argument("--renderer", choices=["sampler", "spectral"], default="sampler",
                    help="Renderer (BASELINE configs: sampler; spectral = SpectralRenderer, SURVEY §8(f) row 2)")
    ap.add_argument("--wave-bands", type=int, default=0, help="SpectralRenderer nWaveBands (default: 32)")
    ap.add_argument("--sampling", choices=["single", "sampler"], default=None,
                    help="SpectralRenderer samplingMethod singleDirection / samplerDirection (default: single)")
    ap.add_argument("--shard", choices=["tiles", "frames"], default="tiles")
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--slices", type=int, default=1, help="tile slices per GPU (single-process --gpus N)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-slices", action="store_true", help="skip the slice_efficiency block")
    ap.add_argument("--serial", action="store_true", help="timed frames in serial mode (profiling runs)")
    ap.add_argument("--bvh", choices=["host", "gpu"], default="host",
                    help="host: the front end's SAH build (node for node the reference's, the default); "
                         "gpu: the linear BVH built on the GPU (pbrtgpu_build_bvh, SURVEY 8(f) row 3)")
    ap.add_argument("--dump-film", default=None, help="rank 0 saves the gathered film (.npy) after the timed steps")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus not in (1, world):
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    threads_mode = world == 1 and args.gpus > 1
    n_gpus = world if world > 1 else args.gpus
    if args.serial:
        os.environ["PBRTGPU_SERIAL"] = "1"
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")          # host-side barrier / max only (no RCCL needed)

    pack, desc = CONFIGS[args.config]
    t_load = time.perf_counter()
    scene = pg.Scene.load(args.scene or os.path.join(ROOT, "scenes", pack), xres=args.res, yres=args.res,
                          spp=args.spp, seed=rank if args.shard == "frames" else 0,
                          integrator=args.integrator, strategy=args.strategy,
                          renderer=None if args.renderer == "sampler" else "spectral", wave_bands=args.wave_bands,
                          sampling=args.sampling)
    if args.integrator != "path":
        desc = desc.replace("path maxdepth", "%s (%s) maxdepth" % (args.integrator, args.strategy or "scene"))
    load_ms = (time.perf_counter() - t_load) * 1e3
    pps = scene.paths_per_sample()
    if args.renderer == "spectral":
        desc += ", SpectralRenderer nWaveBands %d %sDirection (%d paths per camera sample)" % (
            scene.flat.wave_bands, "single" if scene.flat.spectral_sampling == 0 else "sampler", pps)
    info = scene.info()
    tile = (args.tile, args.tile)
    ntx, nty = pg.tile_grid(scene, tile)
    shape = (scene.height, scene.width, scene.bands)

    if threads_mode:
        if pg.gpu_lib().pbrtgpu_device_count() < args.gpus:
            raise SystemExit("--gpus %d: only %d devices visible" % (args.gpus, pg.gpu_lib().pbrtgpu_device_count()))
        devs = [pg.Device(i) for i in range(args.gpus)]
        if args.bvh == "gpu":
            scene = devs[0].build_bvh(scene)
        t_up = time.perf_counter()
        for d in devs:
            d.upload(scene)
        upload_ms = (time.perf_counter() - t_up) * 1e3
        film = np.zeros(shape, np.float32)
        dev, tiles = devs[0], None

        def step():
            _, st = pg.render_multi(devs, tile=tile, slices_per_device=args.slices, out=film)
            return st[:, pg.STAT_PATHS].sum()
    else:
        # one GPU per rank; ranks beyond the visible devices share them (a 1-GPU box running a
        # 2-rank rehearsal of the multi-GPU path)
        dev = pg.Device(local % max(1, pg.gpu_lib().pbrtgpu_device_count()))
        if args.bvh == "gpu":
            scene = dev.build_bvh(scene)
        t_up = time.perf_counter()
        dev.upload(scene)
        upload_ms = (time.perf_counter() - t_up) * 1e3
        if world > 1 and args.shard == "tiles":
            tiles = pg.tile_slice(ntx * nty, rank, world)
            if one_node(world):
                tag = os.environ.get("TORCHELASTIC_RUN_ID", "") + "_" + os.environ.get("MASTER_PORT", "0")
                film_path, film = shared_film(shape, rank, dist, tag)
            else:
                film_path, film = None, np.zeros(shape, np.float32)
        else:
            tiles, film_path = None, None
            film = np.zeros(shape, np.float32)

        def step():
            st = dev.render(tiles=tiles, tile=tile)
            dev.gather(film, tiles=tiles, tile=tile)      # film tiles back on the host
            return st[pg.STAT_PATHS]

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    paths = 0.0
    for _ in range(args.steps):
        paths += step()                  # returns after the film is on the host (device synced)
    elapsed = time.perf_counter() - t0
    my_elapsed = elapsed
    if dist is not None:
        dist.barrier()
    elapsed, total_paths = reduce_over_ranks(dist, elapsed, paths)
    per_rank = None
    if dist is not None:
        import torch
        g = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(g, torch.tensor([my_elapsed], dtype=torch.float64))
        per_rank = [round(float(x[0]) / args.steps * 1e3, 2) for x in g]

    if dist is not None and args.shard == "tiles" and not one_node(world):
        film = compose_film(film, dist)   # multi-node: private films -> rank 0
    if args.dump_film and rank == 0:
        np.save(args.dump_film, np.asarray(film))
    frame_paths = paths / args.steps    # this rank's share of a frame
    roof = None
    if rank == 0 and not args.no_roofline:
        # the profiles/hbm_traffic.json key of this workload (PMC traffic is per integrator / renderer)
        integ_key = {"path": "", "directlighting": "_dl", "metadata": "_meta"}[args.integrator]
        cfg = args.config + integ_key + ("" if args.renderer == "sampler" else "_spec")
        roof = exclusive_roofline(dev, scene, tiles, tile, frame_paths, cfg, pps)

    slices = None
    if rank == 0 and n_gpus == 1 and not threads_mode and args.shard == "tiles" and not args.no_slices:
        slices = slice_efficiency(dev, scene, tile, elapsed / args.steps * 1e3, frame_paths)

    setup = None
    if rank == 0:
        setup = setup_times(dev, scene, args.config, load_ms, upload_ms, args.bvh == "gpu")

    cpu = None
    if rank == 0 and n_gpus == 1 and not args.no_cpu:
        cpu = cpu_baseline(scene, args.cpu_seconds)

    if rank == 0:
        value = total_paths / elapsed / 1e6
        line = {
            "metric": METRIC,
            "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak" if args.shard == "frames" else "strong",
            "vs_baseline": None, "dtype": "f32",
            "data": "packaged scene %s (scene pack built from the reference's scene file), fixed per-path seeds"
                    % pack.replace(".pack", ""),
            "config": {"workload": desc % (scene.bands, info["maxdepth"], scene.spp, scene.width, scene.height),
                       "config": args.config, "paths_per_frame": int(scene.width * scene.height * scene.spp * pps),
                       "shard": args.shard, "tile": args.tile,
                       "parallelism": "%s x%d%s" % ("tiles" if args.shard == "tiles" else "frames", n_gpus,
                                                    " (threads, one process)" if threads_mode else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if setup is not None:
            line["setup_ms"] = setup["total_ms"]
            line["setup"] = setup
        hbm = frame_hbm(roof, args.config, args.integrator, args.renderer, elapsed / args.steps, n_gpus)
        if hbm is not None:
            line["hbm_GBps"] = hbm["GBps"]
            line["hbm"] = hbm
        if slices is not None:
            line["slice_efficiency"] = slices
        if per_rank is not None:
            line["per_gpu_ms_per_step"] = per_rank
        if args.bvh == "gpu":
            line["config"]["bvh"] = "GPU linear BVH (%d nodes): build %.2f ms device, %.2f ms call" % (
                scene.flat.n_nodes, scene.build_ms[0], scene.build_ms[1])
        if args.serial:
            line["note"] = "serial mode (profiling): one lane, no concurrent kernels"
        print(json.dumps(line), flush=True)
    if threads_mode:
        for d in devs:
            d.close()
    else:
        dev.close()
    if dist is not None:
        dist.barrier()
        if rank == 0 and film_path:
            os.unlink(film_path)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
