"""bench.py -- Mpaths/s of the MI355X spectral path tracer on BASELINE.json configs[1].

Workload (N=1): killeroo-simple, SampledSpectrum 32 bands (the reference build's
nSpectralSamples; BASELINE's "30 bands" names the same config), 'path' integrator
maxdepth 5, 700x700 film, 256 spp -> 125.44 M camera paths per step.  One step = one
full-frame render through the C-ABI (pbrtgpu_render_tiles): every path traced, every
sample accumulated into the film in the reference's order.  The scene is uploaded once;
its BVH/meshes stay resident in HBM, so the timed region starts with inputs in HBM.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one process per GPU.
Image tiles / frames shard with no data-path collective.  Default "weak": every rank
renders its own full frame with per-rank seed (fixed per-GPU work);  "--shard tiles"
splits ONE frame's tiles round-robin over ranks (strong).  The only collectives are the
barrier around the timed region and the max-over-ranks of the elapsed time.

Extra JSON fields: "roofline" for the dominant kernel (k_render, the path megakernel)
and "cpu_baseline" (the CPU restatement in oracle/, timed on this host's cores over a
bounded, representative sample of the same workload).  See DESIGN.md §5.
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


def trace_bytes(work, kernel):
    """algorithmic bytes of a traversal kernel = every BVH node it visits
    (32 B), every primitive it tests (48 B pre-gathered triangle, 176 B quadric record),
    plus the ray it reads, the answer it writes and its queue entry."""
    if kernel == "k_trace_closest":
        return (NODE_BYTES * work["nodes_closest"] + TRI_BYTES * work["tris_closest"]
                + QUAD_BYTES * work["quads_closest"] + (RAY_BYTES + HIT_BYTES + QENTRY_BYTES) * work["rays"])
    return (NODE_BYTES * work["nodes_shadow"] + TRI_BYTES * work["tris_shadow"] + QUAD_BYTES * work["quads_shadow"]
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


def cpu_baseline(scene, target_s):
    """CPU restatement (oracle/liboracle.so, TEST INFRASTRUCTURE) on the host cores: all
    samples of pseudo-randomly spread pixels, sized to ~target_s seconds of work."""
    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = max(1, min(16, ncpu))
    o = pg.oracle()
    spp = scene.spp
    probe = 256 * spp // 16 * threads
    t = time.perf_counter()
    o.trace_range(scene, 0, probe, threads)
    dt = time.perf_counter() - t
    count = int(max(probe, probe * target_s / max(dt, 1e-3)))
    count = (count + spp - 1) // spp * spp
    t = time.perf_counter()
    n = o.trace_range(scene, 0, count, threads)
    dt = time.perf_counter() - t
    return {"value": n / dt / 1e6, "unit": "Mpaths/s", "cores": threads, "kind": "port",
            "sample": "%d paths = all %d samples of %d pseudo-randomly spread pixels of the same frame, "
                      "%.1f s on %d threads" % (n, spp, n // spp, dt, threads)}


def shard_tiles(ntiles, rank, world):
    """Tile ids of one rank when ONE frame's tiles are split over ranks (--shard tiles):
    round-robin, so every rank gets a spread of cheap and expensive image regions."""
    return np.arange(rank, ntiles, world, dtype=np.int32)


def reduce_over_ranks(dist, elapsed, paths, device):
    """(max elapsed over ranks, total paths over ranks) -- the only collectives of the run."""
    if dist is None:
        return elapsed, paths
    import torch
    t = torch.tensor([elapsed, paths], dtype=torch.float64, device=device)
    mx = t.clone()
    dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
    dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
    return float(mx[0]), float(t[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "killeroo-simple.pack"))
    ap.add_argument("--res", type=int, default=700)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--shard", choices=["frames", "tiles"], default="frames")
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    scene = pg.Scene.load(args.scene, xres=args.res, yres=args.res, spp=args.spp,
                          seed=rank if args.shard == "frames" else 0)
    info = scene.info()
    dev = pg.Device(local)
    dev.upload(scene)

    tiles = None
    if args.shard == "tiles" and world > 1:
        c = scene.flat.camera
        tw = (c.sx_end - c.sx_start + args.tile - 1) // args.tile
        th = (c.sy_end - c.sy_start + args.tile - 1) // args.tile
        tiles = shard_tiles(tw * th, rank, world)

    def step():
        return dev.render(tiles=tiles, tile=(args.tile, args.tile))

    for _ in range(args.warmup):
        step()

    def sync_all():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    sync_all()
    t0 = time.perf_counter()
    paths = 0.0
    kern = {}
    for _ in range(args.steps):
        st = step()                      # returns after the film is complete (device synced)
        paths += st[pg.STAT_PATHS]
        tm = dev.timing()
        for k in pg.Timing.KERNELS:
            a = kern.setdefault(k, [0.0, 0])
            a[0] += tm[k]["ms"]
            a[1] += tm[k]["launches"]
    elapsed = time.perf_counter() - t0
    sync_all()
    elapsed, total_paths = reduce_over_ranks(dist, elapsed, paths, "cuda")

    # roofline of the dominant kernel: algorithmic bytes (from one instrumented, untimed
    # render of the same frame) / its device time (HIP events around every launch)
    dom = max(("k_trace_closest", "k_trace_shadow", "k_shade"), key=lambda k: kern[k][0])
    dev.render(tiles=tiles, tile=(args.tile, args.tile), count_work=True)
    work = dev.timing()["work"]
    frame_paths = paths / args.steps
    if dom == "k_shade":
        byts = shade_bytes(work, frame_paths, scene.bands)
    else:
        byts = trace_bytes(work, dom)                     # per frame
    sec = kern[dom][0] / args.steps * 1e-3                # per frame
    achieved = byts / sec / 1e9
    launches = kern[dom][1] / args.steps
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": dom,
            "avg_launch_ms": round(kern[dom][0] / max(kern[dom][1], 1), 4),
            "launches_per_step": launches, "alg_bytes_per_launch": round(byts / max(launches, 1)),
            "per_path": {k: round(v / frame_paths, 3) for k, v in work.items()},
            "kernel_ms_per_step": {k: round(v[0] / args.steps, 2) for k, v in kern.items()},
            "kernel_alg_GBps": {
                "k_trace_closest": round(trace_bytes(work, "k_trace_closest") / (kern["k_trace_closest"][0] / args.steps * 1e-3) / 1e9, 1),
                "k_trace_shadow": round(trace_bytes(work, "k_trace_shadow") / (kern["k_trace_shadow"][0] / args.steps * 1e-3) / 1e9, 1),
                "k_shade": round(shade_bytes(work, frame_paths, scene.bands) / (kern["k_shade"][0] / args.steps * 1e-3) / 1e9, 1)},
            # the two wavefront lanes and the shadow stream run kernels concurrently, so the
            # per-kernel event spans above overlap; this is all three kernels' algorithmic
            # bytes of a frame over the wall time of a step
            "pipeline_alg_GBps": round((trace_bytes(work, "k_trace_closest") + trace_bytes(work, "k_trace_shadow")
                                        + shade_bytes(work, frame_paths, scene.bands)) / (elapsed / args.steps) / 1e9, 1)}
    tf = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    if os.path.exists(tf):
        with open(tf) as f:
            tr = json.load(f)
        ent = tr.get(dom)
        if ent and ent.get("res") == args.res and ent.get("spp") == args.spp:
            roof["traffic"] = ent.get("hbm_bytes_per_launch")
            roof["traffic_source"] = tr.get("source")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(scene, args.cpu_seconds)

    if rank == 0:
        value = total_paths / elapsed / 1e6
        line = {
            "metric": "Mpaths/sec (whole node) + HBM GB/s; spectral path tracer at 1/2/4/8 MI355X",
            "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak" if args.shard == "frames" else "strong",
            "vs_baseline": None, "dtype": "f32", "data": "packaged scene killeroo-simple "
            "(scene pack built from the reference's scene file), fixed per-path seeds",
            "config": {"workload": "killeroo-simple SampledSpectrum %d bands, path maxdepth %d, %dspp, %dx%d"
                       % (scene.bands, info["maxdepth"], scene.spp, scene.width, scene.height),
                       "paths_per_step_per_gpu": int(paths / args.steps), "shard": args.shard,
                       "parallelism": "%s x%d" % ("frames" if args.shard == "frames" else "tiles", world)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
