"""Bit-exact rates of the GPU against the reference fixtures and the oracle, per fixture family
(for setting the test thresholds).  Run on the GPU box from the repo root."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pbrtgpu as pg  # noqa: E402
from conftest import GOLDEN  # noqa: E402
import test_oracle_golden as tog  # noqa: E402


def rate(name, scene_fn):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    scene = scene_fn(g, name)
    with pg.Device(0) as d:
        d.upload(scene)
        L = d.trace_paths(g["keys"])
    ref = g["L"]
    same = np.all(L.view(np.int32) == ref.view(np.int32), axis=1)
    rel = np.abs(L - ref).max(axis=1) / np.maximum(np.abs(ref).max(axis=1), 1e-30)
    Lo = pg.oracle().trace_paths(scene, g["keys"])
    so = np.all(L.view(np.int32) == Lo.view(np.int32), axis=1)
    print("%-45s n %6d  exact vs ref %.5f  rel>1e-4 %.5f  exact vs oracle %.6f" %
          (name, len(same), same.mean(), (rel > 1e-4).mean(), so.mean()), flush=True)


for m in tog.SPEC:
    rate(m % "paths", lambda g, n: tog.spec_scene(pg, g, n))
for n in ["killeroo_rgb_paths_48x40s4", "killeroo_rgb_keys_c1_400x400s64"]:
    rate(n, lambda g, n: tog.rgb_scene(pg, g))
