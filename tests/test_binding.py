"""The reference-side binding (integration/gpupathrenderer.{h,cpp}) against
the reference itself: it compiles with the reference's own headers (core/renderer.h:35-46,
film.h, camera.h, paramset.h) and links into the reference harness (oracle/ref/Makefile,
target gpupath) beside the reference's parser, scene objects and camera.  `Renderer "gpupath"`
is created as MakeRenderer's branch would create it; in this container (no GPU) Render must
fail cleanly -- Error(), a status, no file -- never fall back to the CPU."""
import os
import subprocess

import pytest

from conftest import ROOT, REF_SCENES

pytestmark = pytest.mark.reference


@pytest.fixture(scope="module")
def harness():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle", "ref"), "gpupath"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return os.path.join(ROOT, "oracle", "_ref", "b32", "pbrt_ref_harness_gpupath")


def test_gpupath_renderer_without_device_fails_cleanly(pg, harness, tmp_path):
    if pg.gpu_lib().pbrtgpu_device_count() > 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([harness, os.path.join(REF_SCENES, "killeroo-simple.pbrt"), "--res", "16", "16", "--gpupath"],
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stderr
    assert "gpupath: no MI355X device" in r.stderr
    assert "gpupath status -2" in r.stderr          # PBRTGPU_E_NODEVICE
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".dat")]
