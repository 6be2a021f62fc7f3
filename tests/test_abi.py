"""C-ABI boundary checks that need no GPU: both product libraries load, export every
function include/*.h declares, and the ctypes mirror of the flattened-scene structs has
the C layout (checked against a probe compiled from the header with gcc)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

INC = os.path.join(ROOT, "include")


def declared(header):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(pbrt\w+)\s*\(", src, flags=re.M)))


def test_gpu_library_exports_header(pg):
    lib = pg.gpu_lib()
    names = declared("pbrtgpu.h")
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(pg.gpu_symbols()) == names
    assert lib.pbrtgpu_abi_version() == pg.ABI_VERSION


def test_host_library_exports_header(pg):
    lib = pg.host_lib()
    names = declared("pbrthost.h")
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(pg.host_symbols()) == names


def test_no_device_is_an_error_not_a_fallback(pg):
    if pg.gpu_lib().pbrtgpu_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError):
        pg.Device(0)


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "pbrtgpu.h"
#define S(t) printf(#t " %zu\n", sizeof(t))
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f))
int main(void) {
  S(pbrtgpu_bvh_node); S(pbrtgpu_prim); S(pbrtgpu_triangle); S(pbrtgpu_mesh); S(pbrtgpu_quadric);
  S(pbrtgpu_material); S(pbrtgpu_light); S(pbrtgpu_light_shape); S(pbrtgpu_camera); S(pbrtgpu_flat_scene);
  S(pbrtgpu_render_desc); S(pbrtgpu_timing);
  O(pbrtgpu_flat_scene, camera); O(pbrtgpu_flat_scene, nodes); O(pbrtgpu_flat_scene, spectra);
  O(pbrtgpu_camera, px_start); O(pbrtgpu_timing, work);
  return 0;
}
"""


def test_struct_layout_matches_header(pg, tmp_path):
    c = tmp_path / "probe.c"
    c.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", INC, str(c), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.split("\n") if l)
    assert int(got["pbrtgpu_flat_scene"]) == ctypes.sizeof(pg.FlatScene)
    assert int(got["pbrtgpu_camera"]) == ctypes.sizeof(pg.Camera)
    assert int(got["pbrtgpu_render_desc"]) == ctypes.sizeof(pg.RenderDesc)
    assert int(got["pbrtgpu_timing"]) == ctypes.sizeof(pg.Timing)
    assert int(got["pbrtgpu_bvh_node"]) == 32
    assert int(got["pbrtgpu_flat_scene.camera"]) == pg.FlatScene.camera.offset
    assert int(got["pbrtgpu_flat_scene.nodes"]) == pg.FlatScene.nodes.offset
    assert int(got["pbrtgpu_flat_scene.spectra"]) == pg.FlatScene.spectra.offset
    assert int(got["pbrtgpu_camera.px_start"]) == pg.Camera.px_start.offset
    assert int(got["pbrtgpu_timing.work"]) == pg.Timing.work.offset
