"""Render one GPU's 1/N interleaved tile slice of a config (as rank 0 of N renders it in
bench.py), `reps` times after one sizing call, and print one JSON line per call: wall ms,
passes and the device time per kernel family (pbrtgpu timing).  A profiling harness for the
slot-pool performance modes: run it under rocprofv3 with PBRTGPU_SLOTS /
PBRTGPU_SLOT_DIV set to compare pool sizes on the same slice.

usage: python tools/slice_run.py [--config c2] [--slice 4] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--slice", type=int, default=4, help="N: render rank 0's 1/N of the tiles (1 = the full frame)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tile", type=int, default=16)
    a = ap.parse_args()
    scene = pg.Scene.load(os.path.join(ROOT, "scenes", CONFIGS[a.config][0]))
    dev = pg.Device(0)
    dev.upload(scene)
    tile = (a.tile, a.tile)
    ntx, nty = pg.tile_grid(scene, tile)
    tiles = pg.tile_slice(ntx * nty, 0, a.slice) if a.slice > 1 else None
    film = np.zeros((scene.height, scene.width, scene.bands), np.float32)
    for r in range(a.reps + 1):   # call 0 sizes the slot pools
        t = time.perf_counter()
        st = dev.render(tiles=tiles, tile=tile)
        t1 = time.perf_counter()
        dev.gather(film, tiles=tiles, tile=tile)
        dt = time.perf_counter() - t
        gms = (time.perf_counter() - t1) * 1e3
        tm = dev.timing()
        print(json.dumps({"config": a.config, "slice": a.slice, "call": r, "ms": round(dt * 1e3, 2),
                          "render_ms": round(dt * 1e3 - gms, 2), "gather_ms": round(gms, 2),
                          "paths": int(st[pg.STAT_PATHS]), "passes": tm["passes"],
                          "Mpaths_s": round(st[pg.STAT_PATHS] / dt / 1e6, 2),
                          "kernel_ms": {k: round(tm[k]["ms"], 2) for k in pg.Timing.KERNELS},
                          "slots": os.environ.get("PBRTGPU_SLOTS"), "slot_div": os.environ.get("PBRTGPU_SLOT_DIV")}),
              flush=True)


if __name__ == "__main__":
    main()
