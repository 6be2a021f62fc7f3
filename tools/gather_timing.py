# Host-side cost of a C2 step outside the kernels: the film read-back (pbrtgpu_film_read /
# _gather into a numpy film) and a 1/8 tile-slice gather, each timed alone after a render
import os, sys, time
import numpy as np
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
scene = pg.Scene.load(os.path.join(R, "scenes", "killeroo-simple.pack"))
ntx, nty = pg.tile_grid(scene, (16, 16))
with pg.Device(0) as d:
    d.upload(scene)
    d.render(spp_end=1)
    film = np.zeros((scene.height, scene.width, scene.bands), np.float32)
    sl = pg.tile_slice(ntx * nty, 0, 8)
    for name, tiles in (("full film read", None), ("1/8 slice gather", sl)):
        ts = []
        for _ in range(5):
            t = time.perf_counter(); d.gather(film, tiles=tiles); ts.append(time.perf_counter() - t)
        print("%s: %.2f ms (min of 5), %.2f ms (mean)" % (name, 1e3 * min(ts), 1e3 * sum(ts) / len(ts)), flush=True)
    ts = []
    for _ in range(3):
        t = time.perf_counter(); d.render(spp_end=1); ts.append(time.perf_counter() - t)
    print("1-spp render call (host setup + 0.5 M paths): %.2f ms (min of 3)" % (1e3 * min(ts)), flush=True)
