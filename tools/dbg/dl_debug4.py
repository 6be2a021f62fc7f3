# scratch: DirectLighting determinism / variant check (debugging aid)
import os, sys
import numpy as np
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(R, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
scene = pg.Scene.load(os.path.join(R, "scenes", "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=2,
                      integrator="directlighting", strategy="all")
c = scene.flat.camera
keys = np.array([(x, y, s) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
                 for s in range(scene.spp)], np.int32)
Lo = pg.oracle().trace_paths(scene, keys)
with pg.Device(0) as d:
    d.upload(scene)
    runs = [d.trace_paths(keys) for _ in range(3)]
for r in runs:
    same = np.all(r.view(np.int32) == Lo.view(np.int32), axis=1)
    print(os.environ.get("TAG", ""), "exact %.4f" % same.mean(), "det", np.array_equal(r, runs[0]), flush=True)
