import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-spectral_amd"))
sys.path.insert(0, ROOT)
REF_SCENES = "/root/reference/scenes"
PACKS = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "reference: needs /root/reference (build container only)")


def pytest_collection_modifyitems(config, items):
    has_ref = os.path.isdir(REF_SCENES)
    for it in items:
        if "reference" in it.keywords and not has_ref:
            it.add_marker(pytest.mark.skip(reason="/root/reference not present"))


@pytest.fixture(scope="session")
def pg():
    import pbrtgpu
    return pbrtgpu


@pytest.fixture(scope="session")
def killeroo64(pg):
    return pg.Scene.load(os.path.join(PACKS, "killeroo-simple.pack"), xres=64, yres=64, spp=4)


@pytest.fixture(scope="session")
def merl_dir(tmp_path_factory):
    """tests/scenes/merl.pbrt next to the synthetic MERL table it names (tools/make_merl.py
    writes the 35 MB table here; it is not committed)."""
    import shutil
    d = tmp_path_factory.mktemp("merl")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_merl
    make_merl.write(str(d / "synthetic.merl"))
    shutil.copy(os.path.join(ROOT, "tests", "scenes", "merl.pbrt"), str(d))
    return str(d)


def merl_scene(pg, merl_dir, cfg):
    w, h, spp, seed, md = [int(v) for v in cfg]
    return pg.Scene.load(os.path.join(merl_dir, "merl.pbrt"), xres=w, yres=h, spp=spp, maxdepth=md, seed=seed)


def bits_equal(a, b):
    """elementwise: the float32 bits are equal, or both values are NaN"""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert a.shape == b.shape, (a.shape, b.shape)
    return (a.view(np.int32) == b.view(np.int32)) | (np.isnan(a) & np.isnan(b))


def assert_bit_exact(got, ref, what=""):
    """every float32 of `got` has the bits of `ref` (NaN as NaN); on failure the message names
    the elements that differ and their largest relative error"""
    same = bits_equal(got, ref)
    if not same.all():
        g64, r64 = np.asarray(got, np.float64), np.asarray(ref, np.float64)
        d = np.abs(g64 - r64)[~same]
        den = np.maximum(np.abs(r64)[~same], 1e-30)
        first = np.argwhere(~same)[:4].tolist()
        raise AssertionError("%s: %d of %d values differ (first %s), max rel %.3e"
                             % (what, int((~same).sum()), same.size, first, float(np.nanmax(d / den))))
