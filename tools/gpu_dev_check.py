"""Quick GPU check: parity on a small render + timing on the C2 configuration."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
pack = os.path.join(ROOT, "scenes", "killeroo-simple.pack")
res = int(sys.argv[1]) if len(sys.argv) > 1 else 700
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
s = pg.Scene.load(pack, xres=res, yres=res, spp=spp)
with pg.Device(0) as d:
    t = time.time(); d.upload(s); print("upload s", time.time() - t, flush=True)
    for it in range(2):
        t = time.time(); st = d.render(); dt = time.time() - t
        print("render wall %.3f s  paths %d  kernel ms %.1f  accum ms %.1f zeroed %d spills %d  Mpaths/s %.2f" % (
            dt, st[0], st[1], st[2], st[3], st[4], st[0] / dt / 1e6), flush=True)
    f = d.film()
    print("film mean", f.mean(), "max", f.max())
