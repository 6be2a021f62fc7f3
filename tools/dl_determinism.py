# DirectLighting determinism + oracle agreement on coverage.pbrt (PBRTGPU_LIB variants)
import os, sys
import numpy as np
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
scene = pg.Scene.load(os.path.join(R, "scenes", "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=3,
                      integrator="directlighting", strategy="all")
c = scene.flat.camera
keys = np.array([(x, y, s) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
                 for s in range(scene.spp)], np.int32)
Lo = pg.oracle().trace_paths(scene, keys)
with pg.Device(0) as d:
    d.upload(scene)
    runs = [d.trace_paths(keys) for _ in range(3)]
ok = all(np.array_equal(r, runs[0]) for r in runs)
ex = min(np.all(r.view(np.int32) == Lo.view(np.int32), axis=1).mean() for r in runs)
print(os.environ.get("PBRTGPU_LIB", "default"), "deterministic", ok, "min exact vs oracle %.5f" % ex, flush=True)
