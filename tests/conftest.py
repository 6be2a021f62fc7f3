import os
import sys

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
