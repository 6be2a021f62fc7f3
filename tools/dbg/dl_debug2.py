# scratch: DirectLighting lost-path hunt (debugging aid)
import os, sys
import numpy as np
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(R, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
PACKS = os.path.join(R, "scenes")
scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=2,
                      integrator="directlighting", strategy="all")
c = scene.flat.camera
keys = np.array([(x, y, s) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
                 for s in range(scene.spp)], np.int32)
Lo = pg.oracle().trace_paths(scene, keys)
def run(tag, ks, env=None):
    for k, v in (env or {}).items(): os.environ[k] = v
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(ks)
        t = d.timing()
    for k in (env or {}): os.environ.pop(k)
    ref = pg.oracle().trace_paths(scene, ks)
    same = np.all(L.view(np.int32) == ref.view(np.int32), axis=1)
    zero = np.all(L == 0, axis=1) & ~np.all(ref == 0, axis=1)
    bad = np.where(~same)[0]
    print("%-28s n %5d exact %.4f ndiff %4d zero %4d passes %d items %s" % (tag, len(ks), same.mean(), len(bad),
          zero.sum(), t["passes"], (bad.min(), bad.max()) if len(bad) else None), flush=True)
run("batch", keys)
run("serial", keys, {"PBRTGPU_SERIAL": "1"})
run("rows 10-16", keys[(keys[:, 1] >= 10) & (keys[:, 1] <= 16)])
run("first 2000", keys[:2000])
run("first 1000", keys[:1000])
run("1000-3000", keys[1000:3000])
run("batch again", keys)
run("batch 4x", np.concatenate([keys] * 4))
