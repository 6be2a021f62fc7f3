# per-GPU step time for 1/N of the C2 frame (what each rank renders at N GPUs)
import os, sys, time
import numpy as np
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
scene = pg.Scene.load(os.path.join(R, "scenes", "killeroo-simple.pack"))
ntx, nty = pg.tile_grid(scene, (16, 16))
tiles = np.arange(ntx * nty, dtype=np.int32)
with pg.Device(0) as d:
    d.upload(scene)
    for n in [int(v) for v in os.environ.get("NS", "1,2,4,8").split(",")]:
        sl = tiles[0::n]
        d.render(tiles=sl)
        ts = []
        for _ in range(3):
            t = time.perf_counter(); st = d.render(tiles=sl); ts.append(time.perf_counter() - t)
        tm = d.timing()
        paths = st[pg.STAT_PATHS]
        print({k: (round(v["ms"], 2), v["launches"]) for k, v in tm.items() if isinstance(v, dict) and "ms" in v})
        print(os.environ.get("PBRTGPU_SLOTS", "default"), "1/%d frame: %.1f ms, %.1f Mpaths/s per GPU, passes %d, x%d = %.0f Mpaths/s ideal" % (
            n, 1e3 * min(ts), paths / min(ts) / 1e6, tm["passes"], n, n * paths / min(ts) / 1e6), flush=True)
