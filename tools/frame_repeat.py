"""GPU box: render one golden frame N times in one process and report, per render, the tiles whose
hash differs from the reference's golden and from the first render (determinism check).
Usage: python3 tools/frame_repeat.py NAME N   (PBRTGPU_LIB selects the library)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pbrtgpu as pg  # noqa: E402
from make_frame_golden import tile_digest  # noqa: E402
from test_frame_golden import _load  # noqa: E402

name, n = sys.argv[1], int(sys.argv[2])
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # > 0: that many samples per pixel (no golden check)
g, scene = _load(pg, name)
if spp:
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
    w, h, _, seed, md, bands, tile = [int(v) for v in g["config"]]
    from test_frame_golden import PACK, _key
    from conftest import PACKS
    scene = pg.Scene.load(os.path.join(PACKS, PACK[_key(name)]), xres=w, yres=h, spp=spp, maxdepth=md, seed=seed)
    g = {"hash": np.zeros(((h + 15) // 16, (w + 15) // 16), np.uint64)}
first = None
good = None
with pg.Device(0) as d:
    d.upload(scene)
    for r in range(n):
        d.render()
        film = d.film()
        hs, sm, _ = tile_digest(film)
        bad = np.argwhere(hs != g["hash"])
        if first is None:
            first = film.copy()
        diff = np.argwhere((film.view(np.uint32) != first.view(np.uint32)).any(axis=2))
        rec = {"name": name, "lib": os.environ.get("PBRTGPU_LIB", ""), "render": r,
               "tiles_vs_golden": [[int(a), int(b)] for a, b in bad[:8]], "n_bad": int(len(bad)),
               "pixels_vs_first": [[int(a), int(b)] for a, b in diff[:8]], "n_pix_diff": int(len(diff))}
        nan = np.argwhere(~np.isfinite(film).all(axis=2))
        if len(nan):   # PBRTGPU_POISON=255: a sample no path wrote reads as NaN
            rec["nonfinite"] = [[int(a), int(b)] for a, b in nan[:8]]
            rec["n_nonfinite"] = int(len(nan))
        if spp:
            bad = []
        if len(bad) == 0 and not spp:
            good = film.copy()
        if spp and good is None:
            good = film.copy()
        elif good is not None:   # the bands of each pixel that differs from a render matching the golden
            px = np.argwhere((film.view(np.uint32) != good.view(np.uint32)).any(axis=2))
            rec["pixels"] = [{"yx": [int(y), int(x)], "bands": [int(k) for k in np.nonzero(film[y, x] != good[y, x])[0]],
                              "rel": [float(v) for v in (film[y, x] - good[y, x]) / np.maximum(np.abs(good[y, x]), 1e-30)]}
                             for y, x in px[:4]]
        print(json.dumps(rec), flush=True)
