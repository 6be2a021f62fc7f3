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
HIT_BYTES = 16 + 3 * (12 + 12 + 8)   # triangle record + 3 vertices (P, N, uv) fetched for shading


def algorithmic_bytes_per_path(st, paths, bands):
    """bytes the path kernel must move per camera path, from the measured
    traversal work (nodes visited, primitive tests, shading fetches) plus the per-sample
    radiance it writes (bands x f32)."""
    b = (NODE_BYTES * st["nodes"] + TRI_BYTES * st["tri_tests"] + QUAD_BYTES * st["quad_tests"]
         + HIT_BYTES * st["hits"]) / float(paths)
    return b + 4.0 * bands


def sample_keys(scene, n, seed=12345):
    """Uniform random (x, y, sample) keys over the frame, for the traversal statistics."""
    c = scene.flat.camera
    rng = np.random.default_rng(seed)
    k = np.empty((n, 3), dtype=np.int32)
    k[:, 0] = rng.integers(c.px_start, c.px_start + c.px_count, n)
    k[:, 1] = rng.integers(c.py_start, c.py_start + c.py_count, n)
    k[:, 2] = rng.integers(0, scene.spp, n)
    return k


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
        tiles = np.arange(rank, tw * th, world, dtype=np.int32)

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
    kms, launches = 0.0, 0
    for _ in range(args.steps):
        st = step()                      # returns after the film is complete (device synced)
        paths += st[pg.STAT_PATHS]
        ms, n = dev.kernel_timing()
        kms += ms * n
        launches += n
    elapsed = time.perf_counter() - t0
    sync_all()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed, paths], dtype=torch.float64, device="cuda")
        mx = t.clone()
        dist.all_reduce(mx[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, total_paths = float(mx[0]), float(t[1])
    else:
        total_paths = paths

    # roofline of the dominant kernel (k_render): algorithmic bytes per launch / avg launch time
    nstat = 1 << 18
    stt = dev.path_stats(sample_keys(scene, nstat))
    bpp = algorithmic_bytes_per_path(stt, nstat, scene.bands)
    avg_ms = kms / max(launches, 1)
    paths_per_launch = paths / max(launches, 1)
    achieved = bpp * paths_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    tf = os.path.join(ROOT, "profiles", "hbm_traffic_k_render.json")
    if os.path.exists(tf):
        with open(tf) as f:
            tr = json.load(f)
        if tr.get("res") == args.res and tr.get("spp_per_launch") == round(paths_per_launch / (args.res * args.res)):
            traffic = tr.get("hbm_bytes_per_launch")

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
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "k_render<%d>" % scene.bands, "avg_launch_ms": round(avg_ms, 3),
                         "launches": launches, "bytes_per_path": round(bpp, 1),
                         "per_path": {k: round(v / nstat, 3) for k, v in stt.items()}},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    dev.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
