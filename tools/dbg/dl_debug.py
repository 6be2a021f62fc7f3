# scratch: DirectLighting GPU vs oracle (debugging aid)
import os, sys
import numpy as np
R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(R, "pbrt-v2-spectral_amd"))
import pbrtgpu as pg
PACKS = os.path.join(R, "scenes")
strategy, md = sys.argv[1], int(sys.argv[2])
scene = pg.Scene.load(os.path.join(PACKS, "coverage.pack"), xres=40, yres=30, spp=4, maxdepth=md,
                      integrator="directlighting", strategy=strategy)
c = scene.flat.camera
print("window", c.sx_start, c.sx_end, c.sy_start, c.sy_end)
keys = np.array([(x, y, s) for y in range(c.sy_start, c.sy_end) for x in range(c.sx_start, c.sx_end)
                 for s in range(scene.spp)], np.int32)
Lo = pg.oracle().trace_paths(scene, keys)
with pg.Device(0) as d:
    d.upload(scene)
    L = d.trace_paths(keys)
    same = np.all(L.view(np.int32) == Lo.view(np.int32), axis=1)
    bad = np.where(~same)[0]
    print("exact", same.mean(), "ndiff", len(bad), "rows", np.unique(keys[bad, 1]), flush=True)
    for i in bad[:6]:
        L1 = d.trace_paths(keys[i:i + 1])
        print("  key", keys[i], "gpu", L[i, :2], "alone", L1[0, :2], "ora", Lo[i, :2])
    # all paths one at a time for a small window
    sel = bad[:40]
    L1 = np.stack([d.trace_paths(keys[i:i + 1])[0] for i in sel])
    print("alone exact", np.all(L1.view(np.int32) == Lo[sel].view(np.int32), axis=1).mean())
    L2 = d.trace_paths(keys[sel])
    print("subset exact", np.all(L2.view(np.int32) == Lo[sel].view(np.int32), axis=1).mean())
