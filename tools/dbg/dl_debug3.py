# scratch: trace one item's DirectLighting steps (PBRTGPU_LIB=lib/exp/dldbg.so)
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
n = int(sys.argv[1])
with pg.Device(0) as d:
    d.upload(scene)
    print("=== batch of", n, flush=True)
    L = d.trace_paths(keys[:n])
    print("passes", d.timing()["passes"], flush=True)
    i = int(os.environ.get("KEY", "1805"))
    print("gpu %a ora %a" % (float(L[i, 0]) if i < len(L) else -1, float(pg.oracle().trace_paths(scene, keys[i:i+1])[0, 0])))
    print("=== alone", flush=True)
    L1 = d.trace_paths(keys[i:i + 1])
    print("alone %a" % float(L1[0, 0]))
